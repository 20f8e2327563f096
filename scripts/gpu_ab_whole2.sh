#!/bin/bash
# Same-process A/B of the whole-file variants (configs[1] and library mixture), then a
# kernel trace of variants 3 and 5 on configs[1] to split leaf vs tree time.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
WV=${WV:-1,3,5,0,4}
timeout -k 10 300 python -u scripts/ab_kernels.py --what whole --files 1000000 --variants $WV --rounds 7 \
    > gpurun_out/ab_small.json 2> gpurun_out/ab_small.err
rc=$?; echo "ab small rc=$rc"; cat gpurun_out/ab_small.json; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what library --files 1250000 --variants $WV --rounds 7 \
    > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib.err
rc=$?; echo "ab lib rc=$rc"; cat gpurun_out/ab_lib.json; if fatal $rc; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ab -o trace \
    -- python3 scripts/ab_kernels.py --what whole --files 1000000 --variants ${TV:-3,5} --rounds 2 --iters 2 \
    > gpurun_out/prof_ab.log 2>&1
rc=$?; echo "trace rc=$rc"
find gpurun_out/prof_ab -name "*kernel_stats.csv" -exec cat {} \;
exit $rc
