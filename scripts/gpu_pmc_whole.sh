#!/bin/bash
# PMC passes (one counter group per run) over the whole-file variants on configs[1] and the
# sampled kernel on configs[2], for VALU busy / instruction counts / bytes per kernel.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
G2="FETCH_SIZE"
i=0
for W in "whole 1" "whole 3" "whole 7" "sampled 21"; do
  set -- $W
  for G in "$G1" "$G2"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmc_w/$1_$2_$i -o pmc \
      -- python3 scripts/ab_kernels.py --what $1 --files 500000 --variants $2 --rounds 1 --iters 1 \
      > gpurun_out/pmc_w_$i.log 2>&1
    rc=$?; echo "pmc $W [$G] rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
python3 scripts/pmc_cmp.py gpurun_out/pmc_w/*
