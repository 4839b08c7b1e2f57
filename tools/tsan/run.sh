#!/bin/bash
# ThreadSanitizer run of the TX queue's lock-free reservation and hand-offs, and of the RX queue's
# double-buffered receive (host code only; the GPU step is stubbed by gpu_stub.cpp); with
# SAN=address,undefined also a mutation fuzz of the pcap reader (fcs_pcap.cpp). Exits non-zero on a sanitizer report or a lost/duplicated frame.
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
# the RX queue (fcs_rxq.cpp) over a socketpair: every good frame once and in order, drop counters
# exact; with STUB_FAIL_EVERY the stubbed GPU check fails every 3rd call (the recovery paths)
g++ -std=c++17 -O1 -g -fsanitize="$SAN" -fno-sanitize-recover=all -I"$ROOT/include" \
    "$HERE/rxq_stress.cpp" "$HERE/gpu_stub.cpp" "$ROOT/nstack_amd/csrc/fcs_rxq.cpp" \
    "$ROOT/nstack_amd/csrc/fcs_host_crc.cpp" -o "${OUT}_rx" -lpthread
for f in 0 3; do
  for c in "1 -1" "7 -1" "64 -1" "64 0" "4096 0" "64 100000000" "7 -2" "64 -2"; do
    STUB_FAIL_EVERY=$f TSAN_OPTIONS="halt_on_error=1 exitcode=66" ASAN_OPTIONS="detect_leaks=1 exitcode=66" \
      UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" timeout -k 5 300 "${OUT}_rx" $c
  done
done
if [ "$SAN" != thread ]; then   # the pcap reader is single-threaded: memory errors only
  g++ -std=c++17 -O1 -g -fsanitize="$SAN" -fno-sanitize-recover=all -I"$ROOT/include" \
      "$HERE/pcap_fuzz.cpp" "$ROOT/nstack_amd/csrc/fcs_pcap.cpp" -o "${OUT}_pcap" -lpthread
  ASAN_OPTIONS="detect_leaks=1 exitcode=66" UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1" \
    timeout -k 5 300 "${OUT}_pcap" 3000
fi
echo "$SAN: clean"
