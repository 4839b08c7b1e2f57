#!/bin/bash
# Last check of the committed tree: the whole GPU suite and smoke().
set -o pipefail
out=gpurun_out/r3aw; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 $out/tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $out/smoke.log 2>&1; rc=$?
tail -1 $out/smoke.log; exit $rc
