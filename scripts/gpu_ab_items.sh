#!/bin/bash
# Parity of the whole-file variant under test (-k), then the same-process A/B of the
# whole-file variants and a kernel trace of the new one.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread \
    -k "${TK:-items}" > gpurun_out/items_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -6 gpurun_out/items_tests.log; [ $rc -eq 0 ] || exit $rc
WV=${WV:-3,6} TV=${TV:-6} bash scripts/gpu_ab_whole2.sh
