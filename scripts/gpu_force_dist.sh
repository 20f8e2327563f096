#!/bin/bash
# The bench's N > 1 branch on the box's one GPU: torch.distributed.run
# with one rank, the nccl backend (RCCL), and --force-dist, so the process group is up at
# world size 1 and every collective statement of the 8-GPU run executes: ProcessGroupNCCL and
# libsdcas's own RCCL communicator (sd_comm_create) in one process, sd_cas_dedup_mgpu in the
# timed steps, the all-gathers / broadcasts of the parity checks on device tensors,
# sd_split_checksum_mgpu's ncclAllGather, the per-rank with-H2D aggregate.  JSON to
# gpurun_out/force_dist.json.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 ${FORCE_DIST_TIMEOUT:-600} python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
    --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29541} bench.py --gpus 1 --dist-backend nccl --force-dist \
    ${FORCE_DIST_ARGS:-} > gpurun_out/force_dist.json 2> gpurun_out/force_dist.err
rc=$?; echo "force-dist rc=$rc"; tail -5 gpurun_out/force_dist.err; head -c 600 gpurun_out/force_dist.json; echo
exit $rc
