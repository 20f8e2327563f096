#!/bin/bash
# round 5: the pipelined steps with the whole-file kernels on a second, lower-priority stream
# (--hash-streams 2) against one stream (1), ABABAB in separate processes on one box
set -u
mkdir -p gpurun_out/r5zc
ARGS="--no-extras --no-cpu-baseline --config-files 0 --checksum-gib 0 --split-gib 0 --steps 30"
for r in 1 2 3; do
  for v in 1 2; do
    timeout -k 10 300 python3 bench.py $ARGS --hash-streams $v > gpurun_out/r5zc/s$v-$r.json 2> gpurun_out/r5zc/s$v-$r.err || exit $?
    python3 -c "
import json; d=json.loads(open('gpurun_out/r5zc/s$v-$r.json').read().strip().splitlines()[-1]); p=d['steps_pipelined']
print('streams $v round $r', 'value %.2f M step %.3f ms sampled %.3f hash %.3f' % (d['value']/1e6, d['ms_per_step'], p['sampled_ms'], p['hash_ms']),
      'sclk', (d['roofline'].get('clock') or {}).get('sclk_mhz_median'), 'prio', p.get('stream_priority_range'), 'parity', d['parity_sample']['mismatches'], d['parity_full']['mismatches'])"
  done
done
