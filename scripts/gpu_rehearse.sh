#!/bin/bash
# bench at N=1 (serial vs concurrent whole-file kernels), then a 2-rank rehearsal of the
# multi-GPU path on the single GPU of the box (gloo transport for the exchange; RCCL
# cannot run two ranks on one device).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u bench.py --serial --no-cpu-baseline --checksum-gib 0 > gpurun_out/bench_serial.json 2> gpurun_out/bench_serial.err
rc=$?; echo "serial rc=$rc"; cat gpurun_out/bench_serial.json; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --share-gpu --dist-backend gloo --files-per-gpu 400000 \
    --checksum-gib 4 --steps 3 --warmup 1 > gpurun_out/rehearse2.json 2> gpurun_out/rehearse2.err
rc=$?; echo "rehearse rc=$rc"; cat gpurun_out/rehearse2.json; tail -3 gpurun_out/rehearse2.err
exit $rc
