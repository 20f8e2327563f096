#!/bin/bash
# round 3: GPU tests + smoke, the stager probe at 15/16 threads, then bench.py (defaults)
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
bash scripts/gpu_tests.sh
rc=$?; if fatal $rc; then exit $rc; fi
for th in 15 16; do
SWEEP="32:4,32:8" timeout -k 10 300 python -u scripts/stager_cpu_probe.py 200000 $th > gpurun_out/stager_probe_200k_t$th.json 2> gpurun_out/stager_probe_t$th.err
r=$?; echo "stager t$th rc=$r"; cat gpurun_out/stager_probe_200k_t$th.json; if fatal $r; then exit $r; fi
done
cat /sys/fs/cgroup/cpu.stat 2>/dev/null | head -6
bash scripts/gpu_bench.sh
rc2=$?
[ $rc -eq 0 ] && exit $rc2
exit $rc
