#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench.  Stops at the first step that
# times out, aborts or crashes (exit 124/134/137/139); a plain test failure still lets
# the bench run so one call yields both.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -5 gpurun_out/gpu_tests.log
if fatal $rc; then exit $rc; fi

timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if fatal $rc; then exit $rc; fi

timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
exit $rc
