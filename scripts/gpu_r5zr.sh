#!/bin/bash
# round 5 final: GPU tests + smoke + default bench (gpu_r5q.sh), then the 8-rank launcher
# rehearsal on the one GPU (gloo, 2-thread host share per rank). Outputs: gpurun_out/r5zr
set -u
bash scripts/gpu_r5q.sh r5zr || exit $?
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u bench.py --gpus 8 --share-gpu --dist-backend gloo --files-per-gpu 300000 \
    --checksum-gib 8 --split-gib 8 --steps 3 --warmup 1 > gpurun_out/r5zr/rehearse8.json 2> gpurun_out/r5zr/rehearse8.err
rc=$?; echo "rehearse8 rc=$rc"
exit $rc
