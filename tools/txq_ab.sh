#!/bin/bash
# One-box A/B of the TX call-site rates (tools/txq_bench) between the product library and another
# build of it (measurement tool): alternating runs, the other library through LD_LIBRARY_PATH
# (txq_bench's RUNPATH names nstack_amd/).
#   bash tools/txq_ab.sh OTHER_LIB_DIR [rounds]
set -e
OTHER=$1; R=${2:-3}
for r in $(seq 1 "$R"); do
  for args in "1 400000 1500 4096 0 null async" "4 200000 1500 4096 0 null async" "16 20000 1500 1024 0 null txq"; do
    echo "product $args $(timeout -k 10 120 tools/txq_bench $args)"
    echo "other   $args $(LD_LIBRARY_PATH=$OTHER timeout -k 10 120 tools/txq_bench $args)"
  done
done
