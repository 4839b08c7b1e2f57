#!/bin/bash
# The batched, FCS-checked RX call site against the reference's per-frame ether_receive, one box,
# one binary (tools/rxq_bench.c): the reference's body (recvfrom per frame, no FCS check), the queue
# without a check, and the queue checking every frame's FCS with the GPU minimum at 0 (every batch
# on the GPU), the default, and a scan; 1500-B and 46-B payloads; recvmmsg batches of 16 and 64.
#   bash tools/rxq_vs_reference.sh OUT.jsonl
set -o pipefail
out=${1:?usage: rxq_vs_reference.sh OUT.jsonl}
: > "$out"
B=tools/rxq_bench
run() { timeout -k 10 120 $B "$@" >> "$out" || { echo "rxq_bench $* failed"; exit 1; }; }
for pay in 1500 46; do
  run 400000 $pay 1 0 reference
  for mb in 16 64; do
    run 400000 $pay $mb 0 queue
    for hm in 0 16384 65536 262144 1048576; do run 400000 $pay $mb 1 queue $hm; done
  done
done
echo "wrote $(wc -l < "$out") lines to $out"
