#!/bin/bash
# round 5, first GPU call: the GPU tests, then the two N > 1 launches VERDICT r4 asks for:
#  (1) bench.py --gpus 2 through its own launcher (no WORLD_SIZE: it starts
#      torch.distributed.run as a child), two ranks sharing the GPU over gloo;
#  (2) the N > 1 branch at world 1 over nccl (--force-dist) with the host budget forced to
#      2 threads -- one rank's share of an 8-GPU node's 16-CPU quota -- with the per-leg
#      wall times of the line's `timing`.
set -u
mkdir -p gpurun_out/r5a
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r5a/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r5a/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u bench.py --gpus 2 --share-gpu --dist-backend gloo --files-per-gpu 400000 \
    > gpurun_out/r5a/rehearse2_launcher.json 2> gpurun_out/r5a/rehearse2_launcher.err
rc=$?; echo "rehearse rc=$rc"; tail -3 gpurun_out/r5a/rehearse2_launcher.err
if fatal $rc; then exit $rc; fi
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 1 --dist-backend nccl --force-dist --host-cpu-budget 2 \
    > gpurun_out/r5a/force_dist_budget2.json 2> gpurun_out/r5a/force_dist_budget2.err
rc2=$?; echo "force-dist budget 2 rc=$rc2"; tail -3 gpurun_out/r5a/force_dist_budget2.err
[ $rc -eq 0 ] && exit $rc2
exit $rc
