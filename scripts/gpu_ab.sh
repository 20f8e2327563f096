#!/bin/bash
# parity tests, then the sampled-kernel A/B, then the bench
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/gpu_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u scripts/ab_kernels.py --what ${AB_WHAT:-sampled} --variants ${AB_VARIANTS:-10,11,20,21,40,41} > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.json; tail -3 gpurun_out/ab.err; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
