#!/bin/bash
# round 5: the 8-rank run's orchestration on one GPU through bench.py's own launcher --
# 8 processes (LOCAL_WORLD_SIZE 8: a host budget of 2 threads each under the box's 16-CPU
# quota), gloo process group, torch dedup transport, split checksum through host memory;
# smaller per-rank shards so eight ranks fit one device.  Every parity check runs; the
# line's `timing` gives the wall time per leg.
set -u
mkdir -p gpurun_out/r5i
timeout -k 10 900 python3 -u bench.py --gpus 8 --share-gpu --dist-backend gloo --files-per-gpu 300000 \
    --checksum-gib 8 --split-gib 8 --steps 5 --warmup 1 \
    > gpurun_out/r5i/rehearse8_launcher.json 2> gpurun_out/r5i/rehearse8_launcher.err
rc=$?; echo "rehearse8 rc=$rc"; tail -3 gpurun_out/r5i/rehearse8_launcher.err; head -c 400 gpurun_out/r5i/rehearse8_launcher.json; echo
exit $rc
