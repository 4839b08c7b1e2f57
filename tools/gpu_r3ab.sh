#!/bin/bash
# Bench line with median-of-3 host-inclusive timings.
set -o pipefail
out=gpurun_out/r3ab; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python3 bench.py > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; exit $rc
