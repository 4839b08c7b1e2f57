# Round-3 re-entry check on the GPU box: GPU suite, IMIX A/B (stream vs flat-only), bench line.
set -o pipefail
out=gpurun_out/r3g; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/gputest.log 2>&1; rc=$?
echo "gputest rc=$rc"; tail -5 $out/gputest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab.py --imix --frames 134217728 --rounds 4 nstack_amd/libnstack_fcs.so tools/variants/libfcs_nostream.so tools/variants/libfcs_streg.so tools/variants/libfcs_stnocrc.so > $out/ab.log 2>&1; rc=$?
echo "ab rc=$rc"; tail -6 $out/ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err; rc=$?
echo "bench rc=$rc"; cat $out/bench.json | head -c 3000; exit $rc
