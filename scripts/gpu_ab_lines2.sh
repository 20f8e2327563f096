#!/bin/bash
# 128-B staged messages: sampled 21 vs 22, library whole_variant 7 vs 8, PMC FETCH_SIZE
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread > gpurun_out/lt2.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/lt2.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what sampled --variants 21,22 --rounds 9 > gpurun_out/ab_s2.json 2> gpurun_out/ab_s2.err
rc=$?; echo "ab sampled rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what whole --variants 7,8 --files 1000000 --rounds 9 > gpurun_out/ab_w2.json 2> gpurun_out/ab_w2.err
rc=$?; echo "ab whole rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what library --variants 7,8 --files 1250000 --rounds 9 --set sampled_variant=22 > gpurun_out/ab_l2.json 2> gpurun_out/ab_l2.err
rc=$?; echo "ab library rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_lines2 -o pmc \
    -- python3 scripts/ab_kernels.py --what library --variants 7,8 --files 1250000 --rounds 1 --iters 1 > gpurun_out/pmc_lines2.log 2>&1
rc=$?; echo "pmc rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_lines3 -o pmc \
    -- python3 scripts/ab_kernels.py --what sampled --variants 21,22 --rounds 1 --iters 1 > gpurun_out/pmc_lines3.log 2>&1
rc=$?; echo "pmc rc=$rc"
python3 - <<'PY'
import json
for f in ("gpurun_out/ab_s2.json", "gpurun_out/ab_w2.json", "gpurun_out/ab_l2.json"):
    d = json.load(open(f))
    print(d["what"], {k: (round(v["median_ms"], 3), round(v["min_ms"], 3), round(v["Tops"], 2)) for k, v in d["variants"].items()})
PY
exit $rc
