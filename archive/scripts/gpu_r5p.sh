#!/bin/bash
# round 5: the block split with the threads submitting their own windows on the shared-fd
# pool (in-tree) against the calling thread submitting them (ab/libsdcas_callersubmit.so),
# alternated ABAB in separate processes on one box; first the split's GPU tests
set -u
mkdir -p gpurun_out/r5p
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -m gpu \
    -k "concurrent or hybrid_split or cohashed or checksum" > gpurun_out/r5p/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5p/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for v in A B; do
    if [ $v = A ]; then L=$PWD/ab/libsdcas_callersubmit.so; else L=$PWD/spacedrive_amd/libsdcas.so; fi
    SD_CAS_LIB=$L timeout -k 10 300 python3 -u scripts/hybrid_checksum_probe2.py 2 cpu_16,hybrid_6,hybrid_8,hybrid_6_files \
        > gpurun_out/r5p/$v$r.json 2> gpurun_out/r5p/$v$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5p/$v$r.json').read().strip().splitlines()[-1])
print('$v$r', {s: {k: round(x, 1) for k, x in v['median'].items()} for s, v in d.items()})"
  done
done
