#!/bin/bash
# Stream kernel v5 (software-pipelined item loop): parity first, then IMIX A/B against v4 and no-prefetch.
set -o pipefail
out=gpurun_out/r3y; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_windowed.py -x -q --timeout 120 --timeout-method thread > $out/t_stream.log 2>&1; rc=$?
echo "stream tests rc=$rc"; tail -3 $out/t_stream.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py --imix --frames 134217728 --rounds 5 nstack_amd/libnstack_fcs.so tools/variants/libfcs_v4.so tools/variants/libfcs_nopf.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -8; exit $rc
