#!/bin/bash
# GPU parity tests + smoke on the box; stops at the first fatal exit (timeout/abort/crash).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_ARGS:-} \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2"; tail -3 gpurun_out/smoke.log
[ $rc -eq 0 ] && exit $rc2
exit $rc
