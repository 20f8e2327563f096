#!/bin/bash
# Same-box A/B of two builds of libsdcas on the bench step: A = ab/libsdcas_old.so (the
# previous build), B = the in-tree library, alternated ABABAB so both see the same box and
# clock history.  Prints sampled / whole / step ms per run.
set -u
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$PWD/ab/libsdcas_old.so; else L=$PWD/spacedrive_amd/libsdcas.so; fi
    SD_CAS_LIB=$L timeout -k 10 200 python3 bench.py --no-extras --no-cpu-baseline --config-files 0 --checksum-gib 0 \
        --split-gib 0 --steps 30 > gpurun_out/ab_$v$r.json 2> gpurun_out/ab_$v$r.err || exit $?
    python3 -c "
import json,sys; d=json.loads(open('gpurun_out/ab_$v$r.json').read().strip().splitlines()[-1]); k=d['kernels']
print('$v$r', 'sampled %.3f whole %.3f step %.3f value %.1f M' % (k['sampled_ms'], k['whole_ms'], d['ms_per_step'], d['value']/1e6))"
  done
done
