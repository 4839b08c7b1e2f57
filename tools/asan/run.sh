#!/bin/bash
# On the GPU box: the ASan + UBSan host build's driver, then the same driver against the fault-hook
# build with the recovery paths (tools/asan/Makefile builds all of them here).
# Leak checking is off (the HIP runtime keeps its allocations until exit); the shadow gap is left
# unprotected for the HSA runtime's address-space reservations.
set -o pipefail
HERE=$(cd "$(dirname "$0")" && pwd)
ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=1:abort_on_error=0:exitcode=66" \
UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1" \
  timeout -k 10 300 "$HERE/driver" && \
ASAN_OPTIONS="detect_leaks=0:protect_shadow_gap=0:halt_on_error=1:abort_on_error=0:exitcode=66" \
UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1" \
  timeout -k 10 300 "$HERE/driver_faults"
