#!/bin/bash
# round 5: the split's GPU tests on the in-tree build (host-function completion flags), then
# A/B against the caller-submits build, ABABAB in separate processes (4 rounds each)
set -u
mkdir -p gpurun_out/r5s
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 240 --timeout-method thread -m gpu \
    -k "concurrent or hybrid_split or checksum" > gpurun_out/r5s/tests.txt 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r5s/tests.txt
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$PWD/ab/libsdcas_callersubmit.so; else L=$PWD/spacedrive_amd/libsdcas.so; fi
    SD_CAS_LIB=$L timeout -k 10 300 python3 -u scripts/hybrid_checksum_probe2.py 4 cpu_16,hybrid_6 \
        > gpurun_out/r5s/$v$r.json 2> gpurun_out/r5s/$v$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5s/$v$r.json').read().strip().splitlines()[-1])
print('$v$r', {s: (round(v['median']['cpu_16'], 1), round(v['median']['hybrid_6'], 1), round(v['median_over_cpu_16']['hybrid_6'], 3)) for s, v in d.items()})"
  done
done
