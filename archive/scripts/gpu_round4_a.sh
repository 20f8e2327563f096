#!/bin/bash
# round 4, first contact: GPU tests + smoke, the N > 1 branch at world 1 over RCCL
# (scripts/gpu_force_dist.sh), then bench.py with its defaults; stops at the first fatal exit
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_tests.sh
rc=$?; if fatal $rc; then exit $rc; fi
bash scripts/gpu_force_dist.sh
rc2=$?; if fatal $rc2; then exit $rc2; fi
bash scripts/gpu_bench.sh
rc3=$?
[ $rc -eq 0 ] && [ $rc2 -eq 0 ] && exit $rc3
exit 1
