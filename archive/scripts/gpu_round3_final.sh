#!/bin/bash
# round 3 final: GPU tests + smoke, bench.py (defaults), then its rocprofv3 trace and PMC
# passes (scripts/profile.sh, TAG=r3f); stops at the first fatal exit
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_tests.sh
rc=$?; if fatal $rc; then exit $rc; fi
bash scripts/gpu_bench.sh
rc2=$?; if fatal $rc2; then exit $rc2; fi
TAG=r3f bash scripts/profile.sh
rc3=$?
[ $rc -eq 0 ] && [ $rc2 -eq 0 ] && exit $rc3
exit 1
