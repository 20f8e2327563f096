#!/bin/bash
# bench.py, then its rocprofv3 kernel trace and PMC passes (scripts/profile.sh) under TAG
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/bench.err; cat gpurun_out/bench.json
[ $rc -eq 0 ] || exit $rc
TAG=${TAG:-r2} bash scripts/profile.sh
