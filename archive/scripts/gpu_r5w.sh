#!/bin/bash
# round 5: kernel trace of the two k_whole_merge8 builds (per-kernel durations)
set -u
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
mkdir -p gpurun_out/r5w
for v in A B; do
  if [ $v = A ]; then export SD_CAS_LIB=$PWD/ab/libsdcas_m8old.so; else export SD_CAS_LIB=$PWD/spacedrive_amd/libsdcas.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5w/$v -o run -- \
      python3 bench.py --no-extras --no-cpu-baseline --checksum-gib 0 --split-gib 0 --steps 5 --warmup 2 \
      > gpurun_out/r5w/$v.json 2> gpurun_out/r5w/$v.err || exit $?
done
