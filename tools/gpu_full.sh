# Full GPU suite and the graft smoke on one box; output under gpurun_out/$1.
set -o pipefail
out=gpurun_out/${1:-full}; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gputest.log 2>&1; rc=$?
echo "gputest rc=$rc"; tail -5 $out/gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -3 $out/smoke.log; exit $rc
