#!/bin/bash
# Segment kernel: jumbo chunks of up to 32 units (half the work-counter atomics): segment tests, a
# one-process A/B at 9000 B and 65536 B, then the jumbo HBM traffic passes.
set -o pipefail
out=gpurun_out/r3au; mkdir -p $out; export TMPDIR=/tmp
step() {   # tag, timeout, command...
  local tag=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$out/$tag.log"; exit $rc; }; return 0
}
step tests 400 python -u -m pytest tests/test_gpu_segil.py -x -q --timeout 300 --timeout-method thread
tail -1 $out/tests.log
step ab_9000 200 python3 -u tools/ab.py --len 9000 --frames 16777216 --rounds 6 tools/variants/libfcs_wide.so tools/variants/libfcs_c32.so
grep GB/s $out/ab_9000.log
step ab_65536 200 python3 -u tools/ab.py --len 65536 --frames 393216 --rounds 6 tools/variants/libfcs_wide.so tools/variants/libfcs_c32.so
grep GB/s $out/ab_65536.log
step jumbo_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof/jumbo_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
step jumbo_write 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof/jumbo_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
echo done
