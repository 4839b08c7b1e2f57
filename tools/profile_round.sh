#!/bin/bash
# Round profile bundle (GPU box): the plain bench line, then the same command under rocprofv3
# kernel-trace stats (its JSON line and the kernel statistics come from one process), then separate
# PMC passes (FETCH_SIZE, WRITE_SIZE; one counter group per run) for the HBM traffic of the headline
# kernel (64 M x 1518 B), of the IMIX arena-stream kernel (BASELINE configs[2]) and of the 9000-B
# jumbo frames' interleaved segment kernel (configs[3]); last, the N = 2 path rehearsed with two ranks
# on the one GPU (sharded fixed and IMIX configs). Outputs under $1.
set -u
OUT=${1:-gpurun_out/prof}; mkdir -p "$OUT"; export TMPDIR=/tmp
step() {   # tag, timeout, command...
  local tag=$1 lim=$2; shift 2
  timeout -k 10 "$lim" "$@" > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "$tag rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  return 0
}
step bench_plain 400 python3 bench.py
step bench_under_rocprof 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o bench -- python3 bench.py
step pmc_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3
step pmc_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/pmc_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3
step imix_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/imix_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3 --imix --frames 134217728
step imix_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/imix_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --imix --frames 134217728
step jumbo_fetch 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/jumbo_fetch" -o run --pmc FETCH_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
step jumbo_write 300 rocprofv3 --kernel-trace --output-format csv -d "$OUT/jumbo_write" -o run --pmc WRITE_SIZE -- python3 tools/prof_fixed.py --reps 3 --len 9000 --frames 16777216
step rehearsal_2ranks 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --frames-per-gpu 16777216 --imix-frames-per-gpu 33554432 --steps 5 --warmup 2
exit 0
