#!/bin/bash
# line-pair load A/B: sampled variants 21 vs 22 (and 12/42), checksum leaf 0 vs 1, with
# PMC FETCH_SIZE for the HBM traffic of each
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -k "sampled_variants or checksum" > gpurun_out/lt.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/lt.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what sampled --variants 21,22,12,11,42,41 --rounds 7 > gpurun_out/ab_s.json 2> gpurun_out/ab_s.err
rc=$?; echo "ab sampled rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what checksum --variants 0,1 --rounds 7 > gpurun_out/ab_c.json 2> gpurun_out/ab_c.err
rc=$?; echo "ab checksum rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_lines -o pmc \
    -- python3 scripts/ab_kernels.py --what sampled --variants 21,22 --rounds 1 --iters 1 > gpurun_out/pmc_lines_s.log 2>&1
rc=$?; echo "pmc s rc=$rc"; if fatal $rc; then exit $rc; fi
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_lines_c -o pmc \
    -- python3 scripts/ab_kernels.py --what checksum --variants 0,1 --rounds 1 --iters 1 > gpurun_out/pmc_lines_c.log 2>&1
rc=$?; echo "pmc c rc=$rc"
python3 - <<'PY'
import json
for f in ("gpurun_out/ab_s.json", "gpurun_out/ab_c.json"):
    d = json.load(open(f))
    print(d["what"], {k: (round(v["median_ms"], 3), round(v["Tops"], 2)) for k, v in d["variants"].items()})
PY
exit $rc
