#!/bin/bash
# Round profile bundle (GPU box): rocprofv3 kernel-trace stats of the default bench command (its
# JSON line and the kernel statistics come from the same process) and separate PMC passes for the
# HBM traffic of the FCS kernel at the bench workload. Outputs under $1.
set -u
OUT=${1:-gpurun_out/prof}; mkdir -p "$OUT"; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench \
    -- python3 bench.py > "$OUT/bench_under_rocprof.log" 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run --pmc FETCH_SIZE \
    -- python3 tools/prof_fixed.py --reps 3 > "$OUT/pmc_fetch.log" 2>&1
rc=$?; echo "pmc fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run --pmc WRITE_SIZE \
    -- python3 tools/prof_fixed.py --reps 3 > "$OUT/pmc_write.log" 2>&1
rc=$?; echo "pmc write rc=$rc"; exit $rc
