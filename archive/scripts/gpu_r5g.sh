#!/bin/bash
# round 5: sd_checksums' co-hashing from pinned memory vs the CPU path alone, with the
# cgroup's throttling counters (scripts/cohash_checksum_probe.py)
set -u
mkdir -p gpurun_out/r5g
timeout -k 10 600 python3 -u scripts/cohash_checksum_probe.py 3 > gpurun_out/r5g/cohash.json 2> gpurun_out/r5g/cohash.err
rc=$?; echo "cohash rc=$rc"; tail -4 gpurun_out/r5g/cohash.err
exit $rc
