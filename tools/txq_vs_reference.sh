#!/bin/bash
# The batched TX call site against the per-frame ether_send it replaces, one box, one binary
# (tools/txq_bench.c): the reference body with the reference's own compiled ether_fcs
# (oracle/_ref/libref_fcs.so, a baseline leg), the queue with its default GPU minimum, the queue with
# every frame through a batch's GPU step (host_max 0, sync_host 0), fire-and-forget producers, and the library's host CRC per
# frame; then a scan of the GPU minimum for fire-and-forget batches; 1..16 synchronous callers, null and socketpair sinks, 1500-B payloads (1518-B frames).
#   bash tools/txq_vs_reference.sh OUT.jsonl
set -o pipefail
out=${1:?usage: txq_vs_reference.sh OUT.jsonl}
: > "$out"
B=tools/txq_bench
run() { timeout -k 10 120 $B "$@" >> "$out" || { echo "txq_bench $* failed"; exit 1; }; }
for sink in null sock; do
  for p in 1 2 3 4 8 16; do
    m=$((40000 / p)); [ $m -lt 5000 ] && m=5000
    run $p $m 1500 1 0 $sink reference
    run $p $m 1500 1024 0 $sink txq -1
    run $p $m 1500 1024 0 $sink txq 0 0
    run $p $m 1500 1 0 $sink hostcrc
  done
  for p in 1 4 8 16; do
    run $p $((400000 / p)) 1500 4096 0 $sink async -1
    run $p $((400000 / p)) 1500 4096 0 $sink async 0
  done
  run 4 10000 -1 1 0 $sink reference
  run 4 10000 -1 1024 0 $sink txq -1
done
# the GPU minimum for fire-and-forget batches (frames cold in the flusher's cache)
for hm in 0 8192 32768 131072 524288; do
  for p in 1 4; do run $p $((400000 / p)) 1500 4096 0 null async $hm; done
  run 1 400000 64 4096 0 null async $hm
done
echo "wrote $(wc -l < "$out") lines to $out"
