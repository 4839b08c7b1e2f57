#!/bin/bash
# Jumbo segment kernel at 14 / 15 waves per CU with packed 1552-B runs (measurement builds): parity, A/B.
set -o pipefail
out=gpurun_out/r3ag; mkdir -p $out; export TMPDIR=/tmp
NSTACK_FCS_LIB=tools/variants/libfcs_seg15.so timeout -k 10 300 python -u -m pytest tests/test_gpu_segil.py -x -q --timeout 120 --timeout-method thread > $out/t_seg15.log 2>&1; rc=$?
echo "seg15 tests rc=$rc"; tail -2 $out/t_seg15.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u tools/ab.py --len 9000 --frames 16777216 --rounds 5 nstack_amd/libnstack_fcs.so tools/variants/libfcs_seg14.so tools/variants/libfcs_seg15.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -4; exit $rc
