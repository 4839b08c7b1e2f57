#!/bin/bash
# Stream kernel: tap word of boundary-free lanes conflict-free (parity, IMIX A/B vs v4).
set -o pipefail
out=gpurun_out/r3ad; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_windowed.py tests/test_gpu_verify.py -x -q --timeout 120 --timeout-method thread > $out/t_stream.log 2>&1; rc=$?
echo "stream tests rc=$rc"; tail -3 $out/t_stream.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u tools/ab.py --imix --frames 134217728 --rounds 5 nstack_amd/libnstack_fcs.so tools/variants/libfcs_v4.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
