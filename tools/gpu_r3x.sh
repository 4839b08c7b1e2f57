#!/bin/bash
# Round-3 session check: GPU suite, one bench line, counter passes on the IMIX arena-stream kernel.
set -o pipefail
out=gpurun_out/r3x; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
bash tools/pmc.sh $out/pmc --imix --frames 134217728 > $out/pmc.log 2>&1; rc=$?
cat $out/pmc.log; exit $rc
