#!/bin/bash
# round 5, after moving the block split's HIP calls to the calling thread: the split probe,
# the GPU tests + smoke, the default bench
set -u
mkdir -p gpurun_out/r5o
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python3 -u scripts/hybrid_checksum_probe2.py 3 cpu_16,gpu_16,hybrid_4,hybrid_6,hybrid_8,hybrid_6_files \
    > gpurun_out/r5o/hybrid.json 2> gpurun_out/r5o/hybrid.err
rc=$?; echo "hybrid rc=$rc"; tail -2 gpurun_out/r5o/hybrid.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r5o/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r5o/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5o/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r5o/smoke.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r5o/bench.json 2> gpurun_out/r5o/bench.err
rc=$?; echo "bench rc=$rc"; head -c 300 gpurun_out/r5o/bench.json; echo
exit $rc
