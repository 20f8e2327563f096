#!/bin/bash
# round 3: from-files routes A/B (direct / hot-buffer staging / CPU path) with CPU time,
# then the stage bench modes with CPU time per file
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u scripts/files_ab.py 200000 16 5 > gpurun_out/files_ab2.json 2> gpurun_out/files_ab2.err
rc=$?; cat gpurun_out/files_ab2.json; tail -3 gpurun_out/files_ab2.err; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/stage_bench.py 200000 16 0,2,3,5,0,2,3,5 > gpurun_out/stage_bench_cpu.txt 2>&1
rc=$?; grep mode gpurun_out/stage_bench_cpu.txt; exit $rc
