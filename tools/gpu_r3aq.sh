#!/bin/bash
# Generic fixed-length kernel: dispenser kept out of scratch memory (new) vs the round-3 product (base),
# one process per length; then the fixed-length GPU tests on the new build.
set -o pipefail
out=gpurun_out/r3aq; mkdir -p $out; export TMPDIR=/tmp
for spec in "64 268435456" "576 33554432" "1000 20000000" "1400 16000000" "1600 14000000" "3060 7000000" "1518 67108864"; do
  set -- $spec
  echo "== len $1 frames $2"
  timeout -k 10 200 python3 -u tools/ab.py --len $1 --frames $2 --rounds 5 tools/variants/libfcs_base.so tools/variants/libfcs_nodscratch.so > $out/ab_$1.log 2>&1; rc=$?
  grep -E "GB/s|same" $out/ab_$1.log | tail -3; [ $rc -ne 0 ] && exit $rc
done
NSTACK_FCS_LIB=tools/variants/libfcs_nodscratch.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_segil.py tests/test_gpu_verify.py -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $out/tests.log; exit $rc
