#!/bin/bash
# round 5: GPU tests + smoke + the default bench on the current code (outputs: gpurun_out/TAG, default r5q)
set -u
T=${1:-r5q}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/$T/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/$T/smoke.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench rc=$rc"
exit $rc
