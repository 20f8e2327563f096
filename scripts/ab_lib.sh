#!/bin/bash
# Same-box A/B of two builds of libsdcas on the bench: A = $AB_A (default ab/libsdcas_old.so,
# the previous build), B = $AB_B (default the in-tree library), alternated ABABAB so both see
# the same box and clock history.  Every run keeps the bench's oracle checks (parity sample of
# the steps, the configs[1]/[2] samples, configs[3] files 0 and 15).  Prints sampled / whole /
# step ms, configs[1]/[2] ms and checksum GB/s per run; JSON lines in gpurun_out/$AB_TAG/.
set -u
A=${AB_A:-$PWD/ab/libsdcas_old.so}
B=${AB_B:-$PWD/spacedrive_amd/libsdcas.so}
TAG=${AB_TAG:-ab}
ARGS=${AB_ARGS:---no-extras --no-cpu-baseline --config-files 0 --checksum-gib 0 --split-gib 0 --steps 30}
mkdir -p gpurun_out/$TAG
for r in 1 2 3; do
  for v in A B; do
    if [ $v = A ]; then L=$A; else L=$B; fi
    SD_CAS_LIB=$L timeout -k 10 300 python3 bench.py $ARGS > gpurun_out/$TAG/$v$r.json 2> gpurun_out/$TAG/$v$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/$TAG/$v$r.json').read().strip().splitlines()[-1]); k=d['kernels']
c=d.get('configs', {}); ck=d.get('checksum', {})
print('$v$r', 'sampled %.3f whole %.3f step %.3f value %.1f M' % (k['sampled_ms'], k['whole_ms'], d['ms_per_step'], d['value']/1e6),
      ' small %.3f sampled1M %.3f' % (c['small']['kernel_ms'], c['sampled']['kernel_ms']) if c else '',
      ' sclk %s' % ((d['roofline'].get('clock') or {}).get('sclk_mhz_median')),
      ' checksum %.1f GB/s' % ck['GBps'] if ck else '', ' parity', d['parity_sample']['mismatches'])"
  done
done
