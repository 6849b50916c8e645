#!/usr/bin/env bash
# Host-code sanitizer run: the library's host half (BVH builder, scene
# packing/validation incl. the wide-tree builder, OBJ/MTL parser, PNG writer) and the
# CPU oracle built with ASan + UBSan, then the CPU tests that drive them. Runs here on
# the CPU; GPU AddressSanitizer is not available on the MI355X pool.
set -euo pipefail
R="$(cd "$(dirname "$0")/.." && pwd)"
make -s -C "$R/pathtracer-cpp_amd" asan
make -s -C "$R/oracle" asan/liboracle.so
export LD_PRELOAD="$(gcc -print-file-name=libasan.so)"
export ASAN_OPTIONS="detect_leaks=0:abort_on_error=1:allocator_may_return_null=1"
export UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1"
export PT_LIB="$R/pathtracer-cpp_amd/lib/asan/libpt_hip.so"
export PT_ORACLE_LIB="$R/oracle/asan/liboracle.so"
cd "$R"
python3 -m pytest -q -x -m "not gpu" -p no:cacheprovider tests/test_capi.py tests/test_obj.py tests/test_oracle_golden.py "$@"
