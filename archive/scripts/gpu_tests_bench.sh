#!/bin/bash
# GPU tests, then bench.py; stops at the first fatal exit (timeout/abort/crash).
set -u
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_tests.sh
rc=$?
if fatal $rc; then exit $rc; fi
bash scripts/gpu_bench.sh
rc2=$?
[ $rc -eq 0 ] && exit $rc2
exit $rc
