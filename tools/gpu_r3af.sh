#!/bin/bash
# Stream kernel with register loads instead of the LDS-DMA slot (measurement builds): parity, IMIX A/B.
set -o pipefail
out=gpurun_out/r3af; mkdir -p $out; export TMPDIR=/tmp
NSTACK_FCS_LIB=tools/variants/libfcs_streg.so timeout -k 10 200 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_windowed.py -x -q --timeout 120 --timeout-method thread > $out/t_streg.log 2>&1; rc=$?
echo "streg tests rc=$rc"; tail -2 $out/t_streg.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/ab.py --imix --frames 134217728 --rounds 5 nstack_amd/libnstack_fcs.so tools/variants/libfcs_streg.so tools/variants/libfcs_stregnt.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
