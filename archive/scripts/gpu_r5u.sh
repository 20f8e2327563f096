#!/bin/bash
# round 5: non-temporal message loads (SD_MSG_NT=1, ab/libsdcas_nt.so) against the default
# build, ABABAB on one box: the sampled pair, k_whole_items and k_ck_leaf, with the clock
set -u
AB_A=$PWD/spacedrive_amd/libsdcas.so AB_B=$PWD/ab/libsdcas_nt.so AB_TAG=r5u \
AB_ARGS="--no-extras --no-cpu-baseline --config-files 0 --checksum-gib 16 --split-gib 0 --steps 30" \
  bash scripts/ab_lib.sh
