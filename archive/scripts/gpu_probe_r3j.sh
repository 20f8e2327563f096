#!/bin/bash
# round 3: thread scaling of the stager's reads (stage_bench modes 0/2) and open/close
set -u
mkdir -p gpurun_out
timeout -k 10 500 python -u scripts/stage_bench.py 200000 1,2,4,8,16 0,2 > gpurun_out/stage_bench_scaling.txt 2>&1
rc=$?; grep -v "^[0-9]" gpurun_out/stage_bench_scaling.txt | awk '{print $2, $4, $7}' | paste - - - | head -20; exit $rc
