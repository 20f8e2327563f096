#!/bin/bash
# round 5: the co-hash thread count, both from-memory entry points (sd_cas_ids: cohash_probe.py;
# sd_checksums: cohash_checksum_probe.py), interleaved rounds
set -u
mkdir -p gpurun_out/r5h
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python3 -u scripts/cohash_probe.py 300000 3 > gpurun_out/r5h/cohash_cas.json 2> gpurun_out/r5h/cohash_cas.err
rc=$?; echo "cas rc=$rc"; tail -2 gpurun_out/r5h/cohash_cas.json | head -c 1500; echo
if fatal $rc; then exit $rc; fi
timeout -k 10 600 python3 -u scripts/cohash_checksum_probe.py 3 > gpurun_out/r5h/cohash_ck.json 2> gpurun_out/r5h/cohash_ck.err
rc2=$?; echo "ck rc=$rc2"; tail -3 gpurun_out/r5h/cohash_ck.err
[ $rc -eq 0 ] && exit $rc2
exit $rc
