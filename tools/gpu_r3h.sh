# Stream kernel: phase stamps (FCS_STAMPS builds, 1 and 2 chains), parity of the 2-chain build, IMIX A/B.
set -o pipefail
out=gpurun_out/r3h; mkdir -p $out
NSTACK_FCS_LIB=tools/variants/libfcs_ststamps.so timeout -k 10 300 python tools/stamps_stream.py > $out/stamps.log 2>&1; rc=$?
echo "stamps rc=$rc"; grep -v amdgpu.ids $out/stamps.log; [ $rc -ne 0 ] && exit $rc
NSTACK_FCS_LIB=tools/variants/libfcs_st2stamps.so timeout -k 10 300 python tools/stamps_stream.py > $out/stamps2.log 2>&1; rc=$?
echo "stamps2 rc=$rc"; grep -v amdgpu.ids $out/stamps2.log; [ $rc -ne 0 ] && exit $rc
NSTACK_FCS_LIB=tools/variants/libfcs_st2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > $out/st2_tests.log 2>&1; rc=$?
echo "st2 tests rc=$rc"; tail -3 $out/st2_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_nostream.so tools/variants/libfcs_st2.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
