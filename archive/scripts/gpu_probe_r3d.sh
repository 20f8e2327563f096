#!/bin/bash
# round 3: the asm G-mix peak (sd_valu_peak) and the file stager's time split
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -u -c "
import spacedrive_amd as sd
c = sd.default_context(0)
print('sd_valu_peak T lane-ops/s:', [round(c.valu_peak() / 1e12, 2) for _ in range(4)])
" > gpurun_out/valu_peak.txt 2>&1
rc=$?; cat gpurun_out/valu_peak.txt; [ $rc -ne 0 ] && exit $rc
SD_PROFILE_FILES=1 timeout -k 10 300 python -u scripts/stager_cpu_probe.py 200000 16 > gpurun_out/stager_probe_200k_b.json 2> gpurun_out/stager_probe_b.err
rc=$?; echo "stager rc=$rc"; cat gpurun_out/stager_probe_200k_b.json; grep sd_files gpurun_out/stager_probe_b.err | tail -6
exit $rc
