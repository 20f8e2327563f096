#!/bin/bash
# round 3 probes: VALU controls (valu_probe6) and the stager vs the CPU path at 16 threads
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 ./scripts/valu_probe6 > gpurun_out/valu_probe6.txt 2>&1
rc=$?; echo "valu_probe6 rc=$rc"; cat gpurun_out/valu_probe6.txt
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/stager_cpu_probe.py 200000 16 > gpurun_out/stager_probe_200k.json 2> gpurun_out/stager_probe.err
rc=$?; echo "stager 200k rc=$rc"; cat gpurun_out/stager_probe_200k.json; tail -3 gpurun_out/stager_probe.err
exit $rc
