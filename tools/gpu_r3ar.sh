#!/bin/bash
# Wide LDS-DMA kernel (fcs_wide_kernel, 1525..1988 B): its GPU tests, a one-process A/B against the
# round-3 kernels for those lengths (libfcs_base: single / generic / segment kernels), then the whole suite.
set -o pipefail
out=gpurun_out/r3ar; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $out/t_wide.log 2>&1; rc=$?
echo "wide tests rc=$rc"; tail -5 $out/t_wide.log; [ $rc -ne 0 ] && exit $rc
for L in 1525 1530 1536 1537 1600 1700 1800 1900 1949 1950 1988; do
  timeout -k 10 200 python3 -u tools/ab.py --len $L --frames $(( (24 << 30) / L )) --rounds 5 tools/variants/libfcs_base.so tools/variants/libfcs_wide.so > $out/ab_$L.log 2>&1; rc=$?
  echo "== $L"; grep -E "GB/s" $out/ab_$L.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; exit $rc
