#!/bin/bash
# Host-inclusive pipeline trace: where the host thread's time goes per call (fixed 1518 B and IMIX).
set -o pipefail
out=gpurun_out/r3al; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_host.py --rounds 3 tools/variants/libfcs_htrace.so > $out/ab.log 2> $out/trace.log; rc=$?
cat $out/ab.log; grep host_trace $out/trace.log | tail -8; exit $rc
