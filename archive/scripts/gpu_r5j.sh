#!/bin/bash
# round 5, the final code: GPU tests + smoke, the default bench, the N > 1 branch at world 1
# over nccl at a 2-thread host budget (what each rank of an 8-GPU node gets)
set -u
mkdir -p gpurun_out/r5j
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/r5j/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -2 gpurun_out/r5j/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5j/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r5j/smoke.txt
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/r5j/bench.json 2> gpurun_out/r5j/bench.err
rc=$?; echo "bench rc=$rc"; head -c 300 gpurun_out/r5j/bench.json; echo
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
    --master-port 29541 bench.py --gpus 1 --dist-backend nccl --force-dist --host-cpu-budget 2 \
    > gpurun_out/r5j/force_dist_budget2.json 2> gpurun_out/r5j/force_dist_budget2.err
rc=$?; echo "force-dist rc=$rc"
exit $rc
