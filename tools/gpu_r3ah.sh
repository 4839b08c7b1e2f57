#!/bin/bash
# Stream-kernel unit-mix fuzz, then the whole GPU suite.
set -o pipefail
out=gpurun_out/r3ah; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -k fuzz -x -q --timeout 200 --timeout-method thread > $out/t_fuzz.log 2>&1; rc=$?
echo "fuzz rc=$rc"; tail -3 $out/t_fuzz.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; exit $rc
