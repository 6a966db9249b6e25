#!/bin/bash
# Host-code sanitizer runs through the CPU tests (the interpreter is not instrumented; its own allocations are
# not leak-checked):
#   tools/run_sanitized.sh [pytest args]       ASan + UBSan (rspl-slam_amd/asan/librspl.so, `make asan`): native
#       map (window / constraint assembly, outlier removal, write-back), line merge passes, point-line relations,
#       the C API and the BA host staging (HostPool workers, per-part buckets, per-range CSR writes);
#   tools/run_sanitized.sh tsan [pytest args]  ThreadSanitizer (rspl-slam_amd/tsan/librspl.so, `make tsan`): the
#       BA host staging with its worker threads (tests/test_ba_stage.py).
# The sanitizer runtime is preloaded into python.
set -o pipefail
cd "$(dirname "$0")/.."
if [ "$1" = tsan ]; then
  shift
  make -s -C rspl-slam_amd/csrc -j8 tsan || exit 1
  RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.tsan-x86_64.so)
  LD_PRELOAD=$RT TSAN_OPTIONS=halt_on_error=1:report_signal_unsafe=0 RSPL_LIB=tsan/librspl.so \
    python -m pytest tests/test_ba_stage.py -q -p no:cacheprovider "$@"
  exit $?
fi
make -s -C rspl-slam_amd/csrc -j8 asan || exit 1
RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 RSPL_LIB=asan/librspl.so \
  python -m pytest tests/test_map.py tests/test_lines.py tests/test_capi.py tests/test_ba_stage.py -q -p no:cacheprovider "$@"
