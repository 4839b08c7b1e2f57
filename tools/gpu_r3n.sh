# Stream kernel v4 with two chains per chunk: parity, A/B on IMIX and on all-1518 packed frames.
set -o pipefail
out=gpurun_out/r3n; mkdir -p $out; export TMPDIR=/tmp
NSTACK_FCS_LIB=tools/variants/libfcs_st4c2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab.py --imix --frames 134217728 --rounds 3 nstack_amd/libnstack_fcs.so tools/variants/libfcs_st4c2.so tools/variants/libfcs_nostream.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -3; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab.py --imix --mix 1518:1 --frames 67108864 --rounds 3 nstack_amd/libnstack_fcs.so tools/variants/libfcs_st4c2.so tools/variants/libfcs_nostream.so > $out/ab1518.log 2>&1; rc=$?
echo "ab1518 rc=$rc"; grep -v amdgpu.ids $out/ab1518.log | tail -3; exit $rc
