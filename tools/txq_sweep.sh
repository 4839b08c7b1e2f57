#!/bin/bash
# TX call-site rates on one GPU box (tools/txq_bench.c): sync producers, fire-and-forget
# producers, and the per-frame drop-in for comparison. Args: producers frames payload max_batch
# linger_usec sink mode.
set -e
B=tools/txq_bench
for args in "1 20000 1500 1024 0 null txq" "4 20000 1500 1024 0 null txq" "16 20000 1500 1024 0 null txq" \
            "16 20000 -1 1024 0 null txq" "16 20000 1500 1024 0 sock txq" \
            "1 400000 1500 4096 0 null async" "2 400000 1500 4096 0 null async" "4 200000 1500 4096 0 null async" "8 200000 1500 8192 0 null async" "8 200000 1500 8192 50 null async" \
            "8 200000 1500 8192 0 sock async" "8 200000 -1 8192 0 null async" "16 100000 1500 8192 0 null async" \
            "1 5000 1500 1 0 null dropin" "4 5000 1500 1 0 null dropin" "16 2000 1500 1 0 null dropin"; do
  timeout -k 10 120 $B $args
done
