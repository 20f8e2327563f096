#!/bin/bash
# bench.py on the box (default flags unless BENCH_ARGS), JSON to gpurun_out/bench.json
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; head -c 600 gpurun_out/bench.json; echo
exit $rc
