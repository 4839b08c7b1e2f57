#!/bin/bash
# Dispenser tail chunks in whole multiples of cmin (segment kernel: unit pairs = 32-B result sectors):
# the kernels' GPU tests, a one-process A/B for 9000 B and 1518 B, then HBM traffic passes.
set -o pipefail
out=gpurun_out/r3at; mkdir -p $out; export TMPDIR=/tmp
step() {   # tag, timeout, command...
  local tag=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$out/$tag.log"; exit $rc; }; return 0
}
step tests 400 python -u -m pytest tests/test_gpu_segil.py tests/test_gpu_dma.py tests/test_gpu_wide.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread
tail -1 $out/tests.log
step ab_9000 200 python3 -u tools/ab.py --len 9000 --frames 16777216 --rounds 6 tools/variants/libfcs_wide.so tools/variants/libfcs_sector.so
grep GB/s $out/ab_9000.log
step ab_1518 200 python3 -u tools/ab.py --len 1518 --frames 67108864 --rounds 6 tools/variants/libfcs_wide.so tools/variants/libfcs_sector.so
grep GB/s $out/ab_1518.log
step jumbo_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof/jumbo_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
step jumbo_write 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof/jumbo_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
step pmc_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof/pmc_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3
step pmc_write 300 rocprofv3 --kernel-trace --output-format csv -d "$out/prof/pmc_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3
echo done
