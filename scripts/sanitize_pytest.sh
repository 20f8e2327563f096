#!/bin/bash
# The non-GPU pytest suite against libsdcas.so built with ASan + UBSan on its host side
# (make -C spacedrive_amd/csrc asan-lib), clang's ASan runtime preloaded into python.
# Log: profiles/r5/sanitize_pytest_asan.txt (SAN_LOG).  (The standalone TSan run is `make sanitize`.)
set -u
cd "$(dirname "$0")/.."
make -s -C spacedrive_amd/csrc asan-lib || exit 1
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
LOG=${SAN_LOG:-profiles/r5/sanitize_pytest_asan.txt}
export SD_CAS_LIB=$PWD/build/csrc/asan/libsdcas_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:alloc_dealloc_mismatch=0
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
{ echo "libsdcas: $SD_CAS_LIB"; echo "runtime: $RT"; echo "ASAN_OPTIONS=$ASAN_OPTIONS UBSAN_OPTIONS=$UBSAN_OPTIONS"; } > $LOG
LD_PRELOAD=$RT${LD_PRELOAD:+:$LD_PRELOAD} python -c "import spacedrive_amd as sd; sd.cpu.blake3(b'x'); print('loaded:', sorted({l.split()[-1] for l in open('/proc/self/maps') if 'sdcas' in l or 'asan' in l}))" >> $LOG 2>&1
LD_PRELOAD=$RT${LD_PRELOAD:+:$LD_PRELOAD} timeout 1200 python -m pytest tests -q -x -m "not gpu" -p no:cacheprovider >> $LOG 2>&1
rc=$?
echo "pytest rc=$rc" >> $LOG
tail -5 $LOG
exit $rc
