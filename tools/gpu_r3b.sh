set -o pipefail
mkdir -p gpurun_out/r3b
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r3b/stream.log 2>&1; rc=$?
echo "stream tests rc=$rc"; tail -30 gpurun_out/r3b/stream.log
exit $rc
