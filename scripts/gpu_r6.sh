#!/bin/bash
# round 6: GPU tests + smoke, the default bench (compact line + full record), then the
# 8-rank launcher rehearsal on the one GPU (gloo, 2-thread host share per rank) through the
# same emitter.  Outputs: gpurun_out/$1/.  Stops at the first failing step.
set -u
T=${1:-r6}
mkdir -p gpurun_out/$T
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > gpurun_out/$T/gpu_tests.txt 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -4 gpurun_out/$T/gpu_tests.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/$T/smoke.txt
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_BENCH:-0}" = 1 ] && exit 0
timeout -k 10 300 python -u bench.py --full-out gpurun_out/$T/bench_full.json \
    > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err
rc=$?; echo "bench rc=$rc"; wc -c gpurun_out/$T/bench.json
[ $rc -eq 0 ] || exit $rc
[ "${SKIP_REHEARSE:-0}" = 1 ] && exit 0
timeout -k 10 600 python3 -u bench.py --gpus 8 --share-gpu --dist-backend gloo --files-per-gpu 300000 \
    --checksum-gib 8 --split-gib 8 --steps 3 --warmup 1 --full-out gpurun_out/$T/rehearse8_full.json \
    > gpurun_out/$T/rehearse8.json 2> gpurun_out/$T/rehearse8.err
rc=$?; echo "rehearse8 rc=$rc"; wc -c gpurun_out/$T/rehearse8.json
exit $rc
