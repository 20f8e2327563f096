#!/bin/bash
# Parity of every whole-file variant, then same-process A/B of the variants on
# configs[1] (small files only) and on the library mixture.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "exhaustive or mixture or configs0" > gpurun_out/ab_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/ab_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/ab_kernels.py --what whole --files 1000000 --variants ${WV:-1,3,0,4} --rounds 7 \
    > gpurun_out/ab_small.json 2> gpurun_out/ab_small.err
rc=$?; echo "ab small rc=$rc"; cat gpurun_out/ab_small.json; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what library --files 1250000 --variants ${WV:-1,3,0,4} --rounds 7 \
    > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib.err
rc=$?; echo "ab lib rc=$rc"; cat gpurun_out/ab_lib.json
exit $rc
