#!/bin/bash
# The RX queue's GPU minimum (fcs_rxq_set_host_max) scanned with repeats: every frame checked, 1500-
# and 46-B payloads, recvmmsg batches of 16, 64 and 256, three runs per setting interleaved (the
# socket's reader/writer scheduling moves single runs by about 15 %).
#   bash tools/rxq_host_max_scan.sh OUT.jsonl
set -o pipefail
out=${1:?usage: rxq_host_max_scan.sh OUT.jsonl}
: > "$out"
B=tools/rxq_bench
for rep in 1 2 3; do
  for pay in 1500 46; do
    for mb in 16 64 256; do
      for hm in 0 65536 262144 1048576; do
        timeout -k 10 120 $B 400000 $pay $mb 1 queue $hm >> "$out" || { echo "rxq_bench failed"; exit 1; }
      done
    done
  done
done
echo "wrote $(wc -l < "$out") lines to $out"
