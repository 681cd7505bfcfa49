#!/bin/bash
# Run the CPU test suite (pytest -m "not gpu") against the host-ASan/UBSan build of the library
# (0xfec_amd/_san/lib0xfec_hip_san.so, built by tests/c/build.py): python gets the shared ASan
# runtime preloaded, the package loads the sanitized library through FEC_LIB_PATH. CPU only:
# with no GPU every HIP call fails cleanly and the host code's validation and error paths run.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
RT=$(ls /opt/rocm/lib/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -n1)
python "$ROOT/tests/c/build.py"
cd /tmp
# the ASan runtime goes first in LD_PRELOAD; anything already preloaded stays behind it
LD_PRELOAD="$RT${LD_PRELOAD:+:$LD_PRELOAD}" ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 \
    FEC_LIB_PATH="$ROOT/0xfec_amd/_san/lib0xfec_hip_san.so" \
    python -m pytest "$ROOT/tests" -m "not gpu" -q -p no:cacheprovider "$@"
