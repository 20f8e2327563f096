#!/bin/bash
# round 3: stager destinations (cold vs cache-resident) and thread counts under the box's CPU quota
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cat /sys/fs/cgroup/cpu.max 2>/dev/null
for th in 15 16; do
SWEEP="32:4,32:8" timeout -k 10 300 python -u scripts/stager_cpu_probe.py 200000 $th > gpurun_out/stager_probe_200k_t$th.json 2> gpurun_out/stager_probe_t$th.err
rc=$?; echo "stager t$th rc=$rc"; cat gpurun_out/stager_probe_200k_t$th.json; [ $rc -ne 0 ] && exit $rc
done
grep nr_throttled /sys/fs/cgroup/cpu.stat 2>/dev/null; cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -8
exit 0
