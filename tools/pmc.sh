#!/bin/bash
# Counter passes for the FCS kernel (run on the GPU box). One rocprofv3 process per pass, kernel
# trace + stats only alongside --pmc (no runtime/sys traces). Stops at the first crash/timeout.
# usage: tools/pmc.sh <outdir> [prof_fixed.py args...]
set -u
OUT=${1:-gpurun_out/pmc}; shift || true
ARGS="$@"
mkdir -p "$OUT"
export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run --pmc "$@" \
      -- python3 tools/prof_fixed.py --reps 2 $ARGS > "$OUT/$tag.log" 2>&1
  local rc=$?
  echo "pass $tag rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
[ -n "${PMC_ALL:-}" ] && run p3 FETCH_SIZE
[ -n "${PMC_ALL:-}" ] && run p4 WRITE_SIZE
run p5 SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT
[ -n "${PMC_ALL:-}" ] && run p6 TA_BUSY_avr TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
exit 0
