#!/bin/bash
# round 5: what bounds the validator split -- scripts/ck_host_cost.cpp's
# "bound" legs on the box's host: 16-thread STREAM-like DRAM legs, the split's memory traffic
# with and without the CPU half's hashing, each half alone; JSON lines to gpurun_out/r5c/.
set -u
mkdir -p gpurun_out/r5c
timeout -k 10 600 scripts/ck_host_cost 32 256 2.4 bound > gpurun_out/r5c/ck_host_bound.jsonl 2> gpurun_out/r5c/ck_host_bound.err
rc=$?; echo "bound rc=$rc"; tail -4 gpurun_out/r5c/ck_host_bound.jsonl
exit $rc
