#!/bin/bash
# Wide kernel at two widths: 104-B windows (7 KiB slots, 13 waves) for 1537..1604 B, 128-B above.
# Wide tests, a one-process A/B against the 128-B windows alone (libfcs_no26), then the whole suite.
set -o pipefail
out=gpurun_out/r3av; mkdir -p $out; export TMPDIR=/tmp
cp nstack_amd/libnstack_fcs.so /tmp/libfcs_two_widths.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $out/t_wide.log 2>&1; rc=$?
echo "wide tests rc=$rc"; tail -2 $out/t_wide.log; [ $rc -ne 0 ] && exit $rc
for L in 1537 1550 1580 1600 1604 1605; do
  timeout -k 10 200 python3 -u tools/ab.py --len $L --frames $(( (24 << 30) / L )) --rounds 5 tools/variants/libfcs_no26.so /tmp/libfcs_two_widths.so > $out/ab_$L.log 2>&1; rc=$?
  echo "== $L"; grep -E "GB/s" $out/ab_$L.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $out/tests.log; exit $rc
