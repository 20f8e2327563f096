#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench on the box's single GPU: both ranks share the
# device and exchange over gloo (RCCL refuses two ranks on one device), so this checks the
# orchestration of every N > 1 leg (sharding, dedup exchange, split checksum, max-over-ranks
# timing), not xGMI.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
SD_BENCH_STACKS_AFTER=${SD_BENCH_STACKS_AFTER:-} timeout -k 10 ${REHEARSE_TIMEOUT:-300} python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --share-gpu --dist-backend gloo --files-per-gpu 400000 \
    --checksum-gib 4 --split-gib 4 --steps 3 --warmup 1 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
rc=$?; echo "rehearse rc=$rc"; cat gpurun_out/rehearse2.json; tail -5 gpurun_out/rehearse2.err
exit $rc
