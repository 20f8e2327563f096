#!/bin/bash
# Kernel trace of the A/B script (per-kernel durations of each variant).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_ab -o t \
  -- python3 scripts/ab_kernels.py --what ${WHAT:-whole} --files 1000000 --variants ${WV:-1,3,5} --rounds 2 --iters 2 \
  > gpurun_out/trace_ab.json 2> gpurun_out/trace_ab.err
rc=$?; echo "trace rc=$rc"; exit $rc
