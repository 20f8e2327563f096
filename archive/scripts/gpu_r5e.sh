#!/bin/bash
# round 5: the GPU tests (the split by blocks among them), then the split probe through the
# library: claims by blocks (g GPU slots) vs by whole files, beside the CPU path
set -u
mkdir -p gpurun_out/r5e
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r5e/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r5e/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python3 -u scripts/hybrid_checksum_probe2.py 3 > gpurun_out/r5e/hybrid.json 2> gpurun_out/r5e/hybrid.err
rc=$?; echo "hybrid rc=$rc"; tail -2 gpurun_out/r5e/hybrid.err
exit $rc
