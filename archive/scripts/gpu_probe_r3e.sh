#!/bin/bash
# round 3: the ring stager -- GPU file tests, then the window/ring sweep at 200k files
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "files or file or length or pipe or scan or policy or hashes" > gpurun_out/gpu_tests_files.log 2>&1
rc=$?; echo "file tests rc=$rc"; tail -5 gpurun_out/gpu_tests_files.log; [ $rc -ne 0 ] && exit $rc
SWEEP="4:4,8:4,16:4,32:4,8:8,16:8,32:2" SD_PROFILE_FILES=1 timeout -k 10 400 python -u scripts/stager_cpu_probe.py 200000 16 \
    > gpurun_out/stager_probe_200k_c.json 2> gpurun_out/stager_probe_c.err
rc=$?; echo "stager rc=$rc"; cat gpurun_out/stager_probe_200k_c.json; grep sd_files gpurun_out/stager_probe_c.err | tail -4
cat /sys/fs/cgroup/cpu.max 2>/dev/null; nproc; grep -c processor /proc/cpuinfo
exit $rc
