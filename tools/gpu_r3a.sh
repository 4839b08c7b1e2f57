set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3a/gputest.log 2>&1; rc=$?
echo "gputest rc=$rc"; tail -5 gpurun_out/r3a/gputest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3a/bench.json 2> gpurun_out/r3a/bench.err; rc=$?
echo "bench rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3a/pmc_write -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 > gpurun_out/r3a/pmc_write.log 2>&1; echo "pmc_write rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3a/jumbo_write -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216 > gpurun_out/r3a/jumbo_write.log 2>&1; echo "jumbo_write rc=$?"
