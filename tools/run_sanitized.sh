#!/bin/bash
# ASan + UBSan run of the host C++ (native map: window / constraint assembly, outlier removal, write-back;
# line merge passes, point-line relations) through the CPU tests, against the sanitized build
# (rspl-slam_amd/asan/librspl.so, `make -C rspl-slam_amd/csrc asan`), with the ASan runtime preloaded into
# python (the interpreter is not instrumented; its own allocations are not leak-checked).
set -o pipefail
cd "$(dirname "$0")/.."
make -s -C rspl-slam_amd/csrc -j8 asan || exit 1
RT=$(/opt/rocm/bin/hipcc -print-file-name=libclang_rt.asan-x86_64.so)
LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 \
UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 RSPL_LIB=asan/librspl.so \
  python -m pytest tests/test_map.py tests/test_lines.py tests/test_capi.py -q -p no:cacheprovider "$@"
