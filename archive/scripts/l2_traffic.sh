#!/bin/bash
# L1 -> L2 and L2 request counts per launch of the hashing kernels (one PMC pass), over the
# short bench run of scripts/profile.sh: do the line-pair loads re-fetch lines from L2?
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
PMC_ARGS="--steps 1 --warmup 0 --checksum-steps 1 --no-cpu-baseline --no-extras --config-reps 1 --warm-ms 0"
timeout -s KILL 300 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCC_REQ_sum TCC_HIT_sum TCC_MISS_sum --output-format csv \
    -d gpurun_out/pmc_l2 -o pmc -- python3 bench.py $PMC_ARGS > gpurun_out/pmc_l2.json 2> gpurun_out/pmc_l2.err
rc=$?; echo "pmc l2 rc=$rc"; exit $rc
