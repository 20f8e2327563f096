#!/bin/bash
# round 5: sd_file_checksums' split from the page cache, through the library: the GPU
# route's reader count g and the CPU path's read piece size ("cpu_read_piece_kib"), in
# interleaved rounds on two tmpfs file sets (scripts/hybrid_checksum_probe2.py)
set -u
mkdir -p gpurun_out/r5d
timeout -k 10 900 python3 -u scripts/hybrid_checksum_probe2.py 3 > gpurun_out/r5d/hybrid.json 2> gpurun_out/r5d/hybrid.err
rc=$?; echo "hybrid rc=$rc"; tail -3 gpurun_out/r5d/hybrid.err
exit $rc
