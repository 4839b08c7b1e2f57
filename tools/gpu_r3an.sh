#!/bin/bash
# One plain bench line on the current tree.
set -o pipefail
out=gpurun_out/r3an; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log; exit $rc
