#!/bin/bash
# round 3: GPU tests with private fd tables in the reader pools, then the from-files A/B
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_tests.sh
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u scripts/files_ab.py 200000 16 5 > gpurun_out/files_ab3.json 2> gpurun_out/files_ab3.err
r=$?; cat gpurun_out/files_ab3.json; tail -3 gpurun_out/files_ab3.err
[ $rc -eq 0 ] && exit $r
exit $rc
