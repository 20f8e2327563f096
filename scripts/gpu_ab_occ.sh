#!/bin/bash
# Occupancy A/B of k_whole_items (whole_variant 7) via dynamic LDS per workgroup.
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u scripts/ab_kernels.py --what whole --files 1000000 --set whole_variant=7 \
    --key whole_lds_kb --variants 0,21,24,30,40 --rounds 7 > gpurun_out/ab_occ.json 2> gpurun_out/ab_occ.err
rc=$?; echo "ab occ rc=$rc"; cat gpurun_out/ab_occ.json
exit $rc
