#!/bin/bash
# round 5, final code: the N > 1 branch over RCCL at world 1 with the 8-rank host share
# (--host-cpu-budget 2), then `bench.py --gpus 2` through its own launcher (2 ranks on the
# one GPU over gloo)
set -u
mkdir -p gpurun_out/r5zd
export PYTHONUNBUFFERED=1
FORCE_DIST_ARGS="--host-cpu-budget 2" bash scripts/gpu_force_dist.sh > gpurun_out/r5zd/force_dist.log 2>&1
rc=$?; echo "force-dist rc=$rc"; cp gpurun_out/force_dist.json gpurun_out/r5zd/force_dist_budget2.json
if [ $rc -ne 0 ]; then tail -5 gpurun_out/force_dist.err; exit $rc; fi
timeout -k 10 400 python -u bench.py --gpus 2 --share-gpu --dist-backend gloo --files-per-gpu 400000 \
    --checksum-gib 4 --split-gib 4 --steps 3 --warmup 1 > gpurun_out/r5zd/launcher2.json 2> gpurun_out/r5zd/launcher2.err
rc=$?; echo "launcher --gpus 2 rc=$rc"; head -c 300 gpurun_out/r5zd/launcher2.json; echo
exit $rc
