#!/bin/bash
# Host-inclusive A/B (frame check split over threads, one metadata copy per chunk), its trace,
# then the whole GPU suite.
set -o pipefail
out=gpurun_out/r3am; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u tools/ab_host.py --rounds 5 tools/variants/libfcs_base.so tools/variants/libfcs_new.so > $out/ab.log 2>&1; rc=$?
cat $out/ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -u tools/ab_host.py --rounds 2 tools/variants/libfcs_htrace.so > $out/ab_trace.log 2> $out/trace.log; rc=$?
cat $out/ab_trace.log; grep host_trace $out/trace.log | tail -4; [ $rc -ne 0 ] && exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $out/tests.log; exit $rc
