#!/bin/bash
# round 4: the checksum GPU tests (the shared huge range), then the library-level NUMA A/B
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
PYTEST_ARGS="-k checksum" bash scripts/gpu_tests.sh
rc=$?; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u scripts/numa_lib_probe.py 4 > gpurun_out/numa_lib.json 2> gpurun_out/numa_lib.err
rc2=$?; echo "numa probe rc=$rc2"; tail -6 gpurun_out/numa_lib.err; head -c 1500 gpurun_out/numa_lib.json
[ $rc -eq 0 ] && exit $rc2
exit 1
