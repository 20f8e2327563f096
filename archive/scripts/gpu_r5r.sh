#!/bin/bash
# round 5: A/B of the block split's two HIP-safe designs, ABABAB in separate processes:
# A = the calling thread submits every window (ab/libsdcas_callersubmit.so), B = the
# threads submit their own on the shared-fd pool (in-tree); the split and the CPU path alone
# interleaved inside each process (scripts/hybrid_checksum_probe2.py, 4 rounds)
set -u
mkdir -p gpurun_out/r5r
export PYTHONUNBUFFERED=1
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$PWD/ab/libsdcas_callersubmit.so; else L=$PWD/spacedrive_amd/libsdcas.so; fi
    SD_CAS_LIB=$L timeout -k 10 300 python3 -u scripts/hybrid_checksum_probe2.py 4 cpu_16,hybrid_6 \
        > gpurun_out/r5r/$v$r.json 2> gpurun_out/r5r/$v$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5r/$v$r.json').read().strip().splitlines()[-1])
print('$v$r', {s: (round(v['median']['cpu_16'], 1), round(v['median']['hybrid_6'], 1), round(v['median_over_cpu_16']['hybrid_6'], 3)) for s, v in d.items()})"
  done
done
