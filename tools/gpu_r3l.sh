# Stream kernel v4: unit size 256 / 512 / 1024 (parity of each, one A/B process).
set -o pipefail
out=gpurun_out/r3l; mkdir -p $out; export TMPDIR=/tmp
for v in u256; do
  NSTACK_FCS_LIB=tools/variants/libfcs_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $out/tests_$v.log 2>&1; rc=$?
  echo "tests $v rc=$rc"; tail -3 $out/tests_$v.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_u1024.so tools/variants/libfcs_u256.so tools/variants/libfcs_nostream.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
