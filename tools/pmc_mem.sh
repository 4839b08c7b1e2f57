#!/bin/bash
# Memory-pipeline counters (L1/TA stalls, L2 read latency, L1 TLB) for one library variant.
# usage: tools/pmc_mem.sh <outdir> <lib.so> [prof_fixed.py args]
set -u
OUT=$1; LIB=$2; shift 2; ARGS="$@"
mkdir -p "$OUT"; export TMPDIR=/tmp
tag=$(basename "$LIB" .so); mkdir -p "$OUT/$tag"
i=0
for set in "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" \
           "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_SERIALIZATION_STALL_sum" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TA_TOTAL_WAVEFRONTS_sum" \
           "GRBM_GUI_ACTIVE SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VALU SQ_INSTS_LDS"; do
  i=$((i+1))
  NSTACK_FCS_LIB=$LIB timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag/p$i" -o run \
      --pmc $set -- python3 tools/prof_fixed.py --reps 2 $ARGS > "$OUT/$tag/p$i.log" 2>&1
  rc=$?; echo "$tag pass $i rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
done
python3 tools/pmc_summary.py "$OUT/$tag" > "$OUT/$tag.json"; cat "$OUT/$tag.json"
