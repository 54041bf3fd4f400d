#!/bin/bash
# The CPU test suite with the oracle (the parity checker) built under
# AddressSanitizer + UndefinedBehaviorSanitizer (host code only; GPU
# sanitizers are not available on this pool).  Usage: bash oracle/run_asan_suite.sh [pytest args]
set -e
cd "$(dirname "$0")/.."
make -C oracle asan > /dev/null
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
export KURA_ORACLE_LIB=$PWD/oracle/libkura_oracle_asan.so
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
LD_PRELOAD="$ASAN_RT $UBSAN_RT" python -m pytest tests -q -m "not gpu" -p no:cacheprovider "$@"
