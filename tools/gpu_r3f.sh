set -o pipefail
mkdir -p gpurun_out/r3f
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f/stream.log 2>&1; rc=$?
echo "stream tests rc=$rc"; tail -3 gpurun_out/r3f/stream.log; [ $rc -ne 0 ] && exit $rc
NSTACK_FCS_LIB=tools/variants/libfcs_streg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3f/streg.log 2>&1; rc=$?
echo "streg tests rc=$rc"; tail -3 gpurun_out/r3f/streg.log
timeout -k 10 300 python tools/ab.py --imix --frames 134217728 --rounds 3 tools/variants/libfcs_nostream.so tools/variants/libfcs_stream4.so tools/variants/libfcs_streg.so > gpurun_out/r3f/ab.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/r3f/ab.log
