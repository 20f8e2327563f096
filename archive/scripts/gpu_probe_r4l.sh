#!/bin/bash
# round 4: slot waits asleep (blocking-sync events) vs polling (SD_AB_SPIN=1), in separate
# processes, alternated twice: the co-hashed in-memory checksums, the split file checksums,
# and the co-hashed sd_cas_ids.  SD_AB_SPIN was a temporary switch in sd_api_impl.h, removed
# once this A/B (profiles/r4/r4l_sync_ab/) showed no difference; the script records how it ran
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
for r in 1 2; do
  for mode in block spin; do
    if [ $mode = spin ]; then export SD_AB_SPIN=1; else unset SD_AB_SPIN; fi
    timeout -k 10 240 python -u scripts/shared_range_probe.py 4 2 > gpurun_out/ab_${mode}_${r}_shared.json 2> gpurun_out/ab_${mode}_${r}_shared.err
    rc=$?; echo "$mode $r shared rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${mode}_${r}_shared.err; exit $rc; fi
    timeout -k 10 300 python -u scripts/hybrid_checksum_probe2.py 2 cpu_16,hybrid_4 > gpurun_out/ab_${mode}_${r}_hyb.json 2> gpurun_out/ab_${mode}_${r}_hyb.err
    rc=$?; echo "$mode $r hybrid rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${mode}_${r}_hyb.err; exit $rc; fi
    timeout -k 10 240 python -u scripts/cohash_probe.py 300000 2 > gpurun_out/ab_${mode}_${r}_cohash.json 2> gpurun_out/ab_${mode}_${r}_cohash.err
    rc=$?; echo "$mode $r cohash rc=$rc"; if [ $rc -ne 0 ]; then tail -5 gpurun_out/ab_${mode}_${r}_cohash.err; exit $rc; fi
  done
done
unset SD_AB_SPIN
exit 0
