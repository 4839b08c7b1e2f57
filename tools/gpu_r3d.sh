set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3e/stream.log 2>&1; rc=$?
echo "stream tests rc=$rc"; tail -5 gpurun_out/r3e/stream.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab.py --imix --frames 134217728 --rounds 3 tools/variants/libfcs_nostream.so tools/variants/libfcs_stream3.so tools/variants/libfcs_stnocrc3.so > gpurun_out/r3e/ab.log 2>&1; echo "ab rc=$?"; tail -4 gpurun_out/r3e/ab.log
