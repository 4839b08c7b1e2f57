#!/bin/bash
set -u
OUT=gpurun_out/pmc_dma; mkdir -p $OUT; export TMPDIR=/tmp
run() {
  local tag=$1; shift
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$tag" -o run --pmc "$@" \
      -- python3 tools/prof_fixed.py --reps 2 --frames 16777216 > "$OUT/$tag.log" 2>&1
  local rc=$?; echo "pass $tag rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run p2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD
run p5 SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT
