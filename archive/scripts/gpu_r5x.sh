#!/bin/bash
# round 5: rotr8 as v_perm_b32 (SD_ROTR8_PERM=1, ab/libsdcas_perm8.so) against v_alignbit
# (in-tree), ABABAB on one box: same issue class, measured for the power-capped clock
set -u
AB_A=$PWD/spacedrive_amd/libsdcas.so AB_B=$PWD/ab/libsdcas_perm8.so AB_TAG=r5x \
AB_ARGS="--no-extras --no-cpu-baseline --checksum-gib 16 --split-gib 0 --steps 30" \
  bash scripts/ab_lib.sh
