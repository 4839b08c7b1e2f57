#!/bin/bash
# Effective shader clock per variant: GRBM_GUI_ACTIVE / 8 XCDs / kernel time (MI355X_MICROARCH DVFS).
# usage: tools/clock_probe.sh <outdir> lib1.so lib2.so ...   (PROF_ARGS: extra tools/prof_fixed.py args)
set -u
OUT=$1; shift
mkdir -p "$OUT"; export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(basename "$lib" .so)
  NSTACK_FCS_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$tag" -o run \
     --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS -- python3 tools/prof_fixed.py --reps 3 ${PROF_ARGS:-} > "$OUT/$tag.log" 2>&1
  rc=$?; echo "$tag rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
  python3 - "$OUT/$tag" <<'PY'
import csv, glob, sys, collections
d = sys.argv[1]
rows = list(csv.DictReader(open(glob.glob(d + "/*counter_collection.csv")[0])))
per = collections.defaultdict(dict)
for r in rows:
    if any(k in r["Kernel_Name"] for k in ("fcs_dma_kernel", "fcs_single_kernel", "fcs_kernel<", "fcs_flat_kernel")):
        per[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
        per[r["Dispatch_Id"]]["t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
for k, v in sorted(per.items()):
    clk = v["GRBM_GUI_ACTIVE"] / 8 / v["t"] / 1e9
    print(f"  dispatch {k}: {v['t']*1e3:.3f} ms  clock {clk:.3f} GHz  VALU {v['SQ_INSTS_VALU']:.3e}  LDS {v['SQ_INSTS_LDS']:.3e}")
PY
done
