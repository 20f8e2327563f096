#!/bin/bash
# round 5: k_whole_merge8 with every node CV loaded at once (SD_MERGE8_PRELOAD=1, in-tree)
# -- the GPU tests, then A/B against the one-node-at-a-time merge (ab/libsdcas_m8old.so),
# ABABAB on one box with configs[1] / configs[2] timed
set -u
mkdir -p gpurun_out/r5v
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu \
    > gpurun_out/r5v/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5v/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
AB_A=$PWD/ab/libsdcas_m8old.so AB_B=$PWD/spacedrive_amd/libsdcas.so AB_TAG=r5v \
AB_ARGS="--no-extras --no-cpu-baseline --checksum-gib 0 --split-gib 0 --steps 30" \
  bash scripts/ab_lib.sh
