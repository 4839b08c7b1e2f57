#!/bin/bash
# Round profile bundle (GPU box), in the order that keeps it consistent:
#   1. bench.py under rocprofv3 kernel-trace stats (its JSON line and the kernel statistics come from
#      one process);
#   2. separate PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run) for the HBM traffic of
#      the headline kernel (64 M x 1518 B), of the IMIX arena-stream kernel (BASELINE configs[2]) and
#      of the 9000-B jumbo frames' segment kernel (configs[3]);
#   3. the bundle files (kernel statistics split per stream, PMC traffic summaries) written as they
#      will be committed, and placed under profiles/$TAG/ of this snapshot, so that
#   4. the plain bench line, run last, quotes exactly these files (profile_kernel_ms from the split
#      statistics, roofline.traffic from the PMC summaries);
#   5. the N = 2 and N = 8 paths rehearsed on the one GPU (two / eight ranks).
# Outputs under $1; the bundle (copy it to profiles/$TAG/) under $1/bundle.
#   bash tools/profile_round.sh OUT [TAG]
set -u
OUT=${1:-gpurun_out/prof}; TAG=${2:-r06_final}
B="$OUT/bundle"
mkdir -p "$OUT" "$B"; export TMPDIR=/tmp
step() {   # tag, timeout, command...
  local tag=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "$tag rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
line() { grep '^{"metric"' "$1" | tail -1; }
step bench_under_rocprof 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py
line "$OUT/bench_under_rocprof.log" > "$B/${TAG}_bench_line_under_rocprof.json"
step pmc_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3
step pmc_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3
step imix_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/imix_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3 --imix --frames 134217728
step imix_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/imix_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --imix --frames 134217728
step jumbo_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/jumbo_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
step jumbo_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/jumbo_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
# the bundle, named as committed
step split 60 python3 tools/kernel_stats_split.py "$(find "$OUT/trace" -name '*kernel_trace.csv' | head -1)" "$B/${TAG}_bench_kernel_stats_split.csv"
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' | head -1)" "$B/${TAG}_bench_kernel_stats.csv"
IMIX_ALG=$(python3 -c "import sys; sys.path.insert(0, '.'); import bench; print(int(bench.imix_lengths(134217728).sum(dtype='uint64')))")
step traffic 60 python3 tools/traffic_summary.py "$OUT" "$B/${TAG}_pmc_traffic.json" --kernel fcs_dma_kernel
step traffic_imix 60 python3 tools/traffic_summary.py "$OUT" "$B/${TAG}_pmc_traffic_imix.json" --kernel fcs_stream_kernel \
  --frames 134217728 --len imix --alg "$IMIX_ALG" --meta $((134217728 * 12)) --sub-fetch imix_fetch --sub-write imix_write
step traffic_jumbo 60 python3 tools/traffic_summary.py "$OUT" "$B/${TAG}_pmc_traffic_jumbo.json" --kernel fcs_segw_kernel \
  --frames 16777216 --len 9000 --sub-fetch jumbo_fetch --sub-write jumbo_write
mkdir -p "profiles/$TAG" && cp "$B"/* "profiles/$TAG/"
# the plain line, quoting the bundle just written
step bench_plain 400 python3 bench.py
line "$OUT/bench_plain.log" > "$B/${TAG}_bench_line.json"
step rehearsal_2ranks 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --frames-per-gpu 16777216 --imix-frames-per-gpu 33554432 --host-gib-per-gpu 2 --steps 5 --warmup 2
line "$OUT/rehearsal_2ranks.log" > "$B/${TAG}_bench_2ranks_on_1gpu_rehearsal.json"
step rehearsal_8ranks 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29518 bench.py --gpus 8 --frames-per-gpu 4194304 --imix-frames-per-gpu 8388608 --host-gib-per-gpu 0.5 --steps 5 --warmup 2
line "$OUT/rehearsal_8ranks.log" > "$B/${TAG}_bench_8ranks_on_1gpu_rehearsal.json"
echo "bundle: $(ls "$B" | tr '\n' ' ')"
exit 0
