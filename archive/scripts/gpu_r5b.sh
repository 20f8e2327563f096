#!/bin/bash
# round 5: A/B of the G mix's a + b + m as one v_add3_u32 (A, the in-tree default) against
# two v_add_u32 (B, SD_ADD3_SPLIT=1 in ab/libsdcas_add3split.so), VERDICT r4 item 6: the
# sampled pair and k_whole_items in the bench's steps, configs[1] / configs[2] at 1 M files,
# configs[3] at 16 GiB; each run oracle-checked.
set -u
AB_A=$PWD/spacedrive_amd/libsdcas.so AB_B=$PWD/ab/libsdcas_add3split.so AB_TAG=r5b_add3 \
AB_ARGS="--no-extras --no-cpu-baseline --config-files 1000000 --checksum-gib 16 --split-gib 0 --steps 30" \
    bash scripts/ab_lib.sh
