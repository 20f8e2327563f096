#!/bin/bash
# round 5: the add3 A/B (scripts/gpu_r5b.sh), then the host bandwidth bound legs (gpu_r5c.sh)
set -u
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_r5b.sh
rc=$?; echo "ab rc=$rc"; if fatal $rc; then exit $rc; fi
bash scripts/gpu_r5c.sh
rc2=$?
[ $rc -eq 0 ] && exit $rc2
exit $rc
