#!/bin/bash
# round 5: k_ck_leaf with several blocks per workgroup and their trees packed -- the GPU
# tests on the in-tree build (4-chunk lanes, 2 blocks per 512-lane workgroup), then the
# committed kernel (ab/libsdcas_old.so: 4-chunk lanes, one block per workgroup) against
# ck4x2 (in-tree), ck4x4 and ck8x2, rotated on one box: configs[3] and its mixed set, the
# split path's 32 GiB file, each run oracle-checked (a first pass, r5zk1, compared 16-chunk
# lanes x 4 blocks and 8 x 2 against the committed kernel)
set -u
mkdir -p gpurun_out/r5zk
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -x -v --timeout 120 --timeout-method thread -m gpu \
    > gpurun_out/r5zk/gpu_tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5zk/gpu_tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
ARGS="--no-extras --no-cpu-baseline --config-files 0 --steps 5 --checksum-gib 64 --split-gib 32"
for r in 1 2 3; do
  for v in old ck4x2 ck4x4 ck8x2; do
    if [ $v = ck4x2 ]; then L=$PWD/spacedrive_amd/libsdcas.so; else L=$PWD/ab/libsdcas_$v.so; fi
    SD_CAS_LIB=$L timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/r5zk/$v-$r.json 2> gpurun_out/r5zk/$v-$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5zk/$v-$r.json').read().strip().splitlines()[-1]); c=d['checksum']; o=d['checksum_one_file']
print('$v round $r', 'checksum %.1f GB/s (%.3f ms/file-batch) mixed %.1f one-file %.1f GB/s' % (c['GBps'], c.get('ms', 0) or 0, c['mixed']['GBps'], o['GBps']),
      'sclk', (c['roofline'].get('clock') or {}).get('sclk_mhz_median'), 'parity', c['parity']['mismatches'], c['mixed']['parity']['mismatches'], o['parity']['mismatches'])"
  done
done
