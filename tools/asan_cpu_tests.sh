#!/bin/bash
# The CPU test suite against the host sanitizer builds (`make asan`):
#   1. libsahara_hip.so with ASan + UBSan in its host code (clang runtime preloaded)
#   2. the oracle with ASan + UBSan (gcc runtime preloaded)
#   3. the CLI tests that run on CPU, against bin/sahara_asan
# Usage: tools/asan_cpu_tests.sh [pytest args]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R" && make -j8 asan > /dev/null || exit 1
CLANG_ASAN=$(ls /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so | head -1)
GCC_ASAN=$(gcc -print-file-name=libasan.so)
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
echo "== libsahara_hip host code (clang ASan/UBSan)"
LD_PRELOAD=$CLANG_ASAN SAHARA_HIP_LIB=$R/build/asan/libsahara_hip.so \
    python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider --ignore=tests/test_cli.py "$@" || exit 1
echo "== oracle (gcc ASan/UBSan)"
LD_PRELOAD=$GCC_ASAN ORACLE_LIB=$R/oracle/liboracle_asan.so \
    python3 -m pytest tests -q -m "not gpu" -p no:cacheprovider --ignore=tests/test_cli.py "$@" || exit 1
echo "== CLI (bin/sahara_asan)"
SAHARA_CLI=$R/bin/sahara_asan python3 -m pytest tests/test_cli.py -q -m "not gpu" -p no:cacheprovider "$@" || exit 1
