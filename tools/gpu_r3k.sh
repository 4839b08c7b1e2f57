# Stream kernel v4 (swizzled 4 KiB slots, no LDS atomic, cursor in registers): parity, A/B, stamps.
set -o pipefail
out=gpurun_out/r3k; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_windowed.py -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -15 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_v3.so tools/variants/libfcs_nostream.so tools/variants/libfcs_st4nocrc.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; [ $rc -ne 0 ] && exit $rc
NSTACK_FCS_LIB=tools/variants/libfcs_st4stamps.so timeout -k 10 300 python tools/stamps_stream.py > $out/stamps.log 2>&1; rc=$?
echo "stamps rc=$rc"; grep -v amdgpu.ids $out/stamps.log; exit $rc
