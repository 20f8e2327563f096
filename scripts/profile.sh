#!/bin/bash
# rocprofv3 kernel trace + stats of a bench run, then PMC passes (one counter group per
# run, as MI355X_MICROARCH.md prescribes) over a short bench run whose launch shapes match
# the bench's (scripts/summarize_profiles.py keys the counters by kernel and grid).
# Output under gpurun_out/; `python scripts/summarize_profiles.py $TAG` copies summaries
# into profiles/.
set -u
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${TAG:-r2}
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o trace \
    -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras \
    > gpurun_out/prof_bench_$TAG.json 2> gpurun_out/prof_bench_$TAG.err
rc=$?; echo "trace rc=$rc"; if fatal $rc; then exit $rc; fi
[ "${PMC:-1}" = "1" ] || exit 0
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/calib_$TAG -o calib \
    -- python3 scripts/pmc_calib.py > gpurun_out/calib_$TAG.log 2>&1
rc=$?; echo "calib rc=$rc"; if fatal $rc; then exit $rc; fi
PMC_ARGS="--steps 1 --warmup 0 --checksum-steps 1 --no-cpu-baseline --no-extras --config-reps 1 --warm-ms 0"
for C in FETCH_SIZE WRITE_SIZE "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"; do
  N=$(echo $C | cut -d' ' -f1)
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d gpurun_out/pmc_${TAG}_$N -o pmc \
      -- python3 bench.py $PMC_ARGS > gpurun_out/pmc_${TAG}_$N.json 2> gpurun_out/pmc_${TAG}_$N.err
  rc=$?; echo "pmc $N rc=$rc"; if fatal $rc; then exit $rc; fi
done
exit 0
