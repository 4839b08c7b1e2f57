#!/bin/bash
# Host pipeline depth 2 (product) against 3 chunks in flight, same process; then the depth-3 trace.
set -o pipefail
out=gpurun_out/r3ao; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_host.py --rounds 5 tools/variants/libfcs_new.so tools/variants/libfcs_depth3.so > $out/ab.log 2>&1; rc=$?
cat $out/ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/ab_host.py --rounds 2 tools/variants/libfcs_depth3t.so > $out/ab_trace.log 2> $out/trace.log; rc=$?
cat $out/ab_trace.log; grep host_trace $out/trace.log | tail -4; exit $rc
