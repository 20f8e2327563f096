#!/bin/bash
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
timeout -k 10 300 python -u scripts/ab_kernels.py --what library --files 1250000 --variants 0,1 --rounds 7 > gpurun_out/ab_lib.json 2> gpurun_out/ab_lib.err
rc=$?; echo "ab lib rc=$rc"; cat gpurun_out/ab_lib.json; if fatal $rc; then exit $rc; fi
for V in 0 1; do
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_ab_$V -o pmc \
    -- python3 scripts/ab_kernels.py --what library --files 1250000 --variants $V --rounds 1 --iters 1 > gpurun_out/pmc_ab_$V.log 2>&1
rc=$?; echo "pmc $V rc=$rc"; if fatal $rc; then exit $rc; fi
done
exit 0
