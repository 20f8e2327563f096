#!/bin/bash
# round 4: the CPU path before (ab/old/libsdcas.so, built from 9d30136) and after its batch
# + load changes, alternated in separate processes on one box: file checksums from the page
# cache (CPU path alone and the split) and the cas / checksum host speeds
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then export SD_CAS_LIB=$PWD/ab/old/libsdcas.so; else unset SD_CAS_LIB; fi
    timeout -k 10 300 python -u scripts/hybrid_checksum_probe2.py 2 cpu_16,hybrid_4 > gpurun_out/ab4x_${v}_${r}_hyb.json 2> gpurun_out/ab4x_${v}_${r}_hyb.err
    rc=$?; echo "$v $r hyb rc=$rc"; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 200 python -u scripts/cpu_speed_probe.py > gpurun_out/ab4x_${v}_${r}_cpu.json 2> gpurun_out/ab4x_${v}_${r}_cpu.err
    rc=$?; echo "$v $r cpu rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
unset SD_CAS_LIB
