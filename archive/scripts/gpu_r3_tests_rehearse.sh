#!/bin/bash
# round 3: syscall costs, GPU tests + smoke, then the 2-rank rehearsal of the N > 1 bench
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
gcc -O2 -o /tmp/syscall_probe scripts/syscall_probe.c && /tmp/syscall_probe && /tmp/syscall_probe | tee gpurun_out/syscall_probe.json
bash scripts/gpu_tests.sh
rc=$?; if fatal $rc; then exit $rc; fi
bash scripts/gpu_rehearse.sh
rc2=$?
[ $rc -eq 0 ] && exit $rc2
exit $rc
