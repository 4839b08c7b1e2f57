#!/bin/bash
# ThreadSanitizer run of the TX queue's lock-free reservation and hand-offs (host code only; the
# GPU step is stubbed by gpu_stub.cpp). Exits non-zero on a sanitizer report or a lost/duplicated frame.
#   bash tools/tsan/run.sh            ThreadSanitizer
#   SAN=address,undefined bash tools/tsan/run.sh   AddressSanitizer + UBSan over the same cases
set -eu
SAN=${SAN:-thread}
HERE=$(cd "$(dirname "$0")" && pwd)
ROOT=$(dirname "$(dirname "$HERE")")
OUT=${TMPDIR:-/tmp}/txq_san_${SAN//,/_}
g++ -std=c++17 -O1 -g -fsanitize="$SAN" -fno-sanitize-recover=all -DFCS_TXQ_TSAN -I"$ROOT/include" \
    "$HERE/txq_stress.cpp" "$HERE/gpu_stub.cpp" "$ROOT/nstack_amd/csrc/fcs_txq.cpp" \
    "$ROOT/nstack_amd/csrc/fcs_host_crc.cpp" -o "$OUT" -lpthread
for c in "1 0" "7 0" "7 30" "64 0" "64 3000" "256 30" "512 0" "4096 0" "4096 30" "4096 3000" \
         "1 0 0" "7 30 0" "64 0 0" "256 30 0" "4096 30 0" "64 0 1000000"; do
  TSAN_OPTIONS="halt_on_error=1 exitcode=66" ASAN_OPTIONS="detect_leaks=1 exitcode=66" \
    UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" timeout -k 5 300 "$OUT" $c
done
echo "$SAN: clean"
