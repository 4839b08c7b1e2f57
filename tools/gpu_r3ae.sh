#!/bin/bash
# Stream kernel at 8 / 12 / 14 / 16 waves per CU (IMIX, one process): latency- or throughput-bound?
set -o pipefail
out=gpurun_out/r3ae; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_wg896.so tools/variants/libfcs_wg768.so tools/variants/libfcs_wg512.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; grep -v amdgpu.ids $out/ab.log | tail -5; exit $rc
