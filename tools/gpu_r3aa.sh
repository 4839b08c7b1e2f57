#!/bin/bash
# Host-inclusive paths: current engine vs the one before the two-stream pipeline (c9a2d1c), one process; bench line.
set -o pipefail
out=gpurun_out/r3aa; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 400 python -u tools/ab_host.py --rounds 6 nstack_amd/libnstack_fcs.so tools/variants/libfcs_host0.so > $out/ab_host.log 2>&1; rc=$?
echo "ab_host rc=$rc"; grep -v amdgpu.ids $out/ab_host.log | tail -6; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py > $out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 600 $out/bench.log; exit $rc
