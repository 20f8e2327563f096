#!/bin/bash
# round 4 final, part 2: the 2-rank gloo rehearsal (scripts/gpu_rehearse.sh), then the
# rocprofv3 trace + PMC passes of the final code (scripts/profile.sh, TAG=r4)
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_rehearse.sh
rc=$?; if fatal $rc; then exit $rc; fi
TAG=r4 bash scripts/profile.sh
rc2=$?
[ $rc -eq 0 ] && exit $rc2
exit 1
