#!/bin/bash
# Wide kernel, third width: 120-B windows (7 KiB slots, 13 waves) for 1605..1787 B (at stride = len).
# Wide tests, a one-process A/B against the build without it (libfcs_no30), then the whole suite.
set -o pipefail
out=gpurun_out/r3ax; mkdir -p $out; export TMPDIR=/tmp
cp nstack_amd/libnstack_fcs.so /tmp/libfcs_three_widths.so
timeout -k 10 400 python -u -m pytest tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $out/t_wide.log 2>&1; rc=$?
echo "wide tests rc=$rc"; tail -2 $out/t_wide.log; [ $rc -ne 0 ] && exit $rc
for L in 1605 1650 1700 1750 1787 1788; do
  timeout -k 10 200 python3 -u tools/ab.py --len $L --frames $(( (24 << 30) / L )) --rounds 5 tools/variants/libfcs_no30.so /tmp/libfcs_three_widths.so > $out/ab_$L.log 2>&1; rc=$?
  echo "== $L"; grep -E "GB/s" $out/ab_$L.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?
tail -1 $out/smoke.log; exit $rc
