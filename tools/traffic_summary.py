#!/usr/bin/env python3
"""Write profiles/<round>_pmc_traffic.json from tools/profile_round.sh's PMC passes.

    python tools/traffic_summary.py gpurun_out/prof profiles/r01_pmc_traffic.json

HBM bytes per launch of the product's fixed-length kernel at the bench workload, corrected as
MI355X_MICROARCH.md's HBM section prescribes: FETCH_SIZE (KB) x 2 on gfx950 for wide streaming
reads, WRITE_SIZE (KB) as is, KB = 1024 B. bench.py reads the file for roofline.traffic.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(outdir, counter, kernel):
    vals, ms = {}, []
    for p in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
                vals[r["Dispatch_Id"]] = vals.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    for p in glob.glob(os.path.join(outdir, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"]:
                ms.append(round((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, 3))
    return (sum(vals.values()) / len(vals) if vals else None), len(vals), ms


def main():
    src, dst = sys.argv[1], sys.argv[2]
    kernel = "fcs_single_kernel"
    frames, L = 64 << 20, 1518
    fetch, n_f, ms_f = per_dispatch(os.path.join(src, "pmc_fetch"), "FETCH_SIZE", kernel)
    write, n_w, ms_w = per_dispatch(os.path.join(src, "pmc_write"), "WRITE_SIZE", kernel)
    alg = frames * L
    rd = fetch * 1024 * 2
    wr = write * 1024
    rec = {
        "round": int(os.path.basename(dst)[1:3]),
        "kernel": "fcs::fcs_single_kernel (fixed length, single segment; product kernel for 1518 B)",
        "frames": frames, "len": L, "algorithmic_bytes_per_launch": alg,
        "command": "tools/profile_round.sh: rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -- "
                   "python3 tools/prof_fixed.py --reps 3 (and a separate --pmc WRITE_SIZE pass)",
        "FETCH_SIZE_kb_per_launch": fetch, "WRITE_SIZE_kb_per_launch": write,
        "correction": "MI355X_MICROARCH.md HBM: on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide "
                      "coalesced read -> x2; WRITE_SIZE taken as is; KB = 1024 B",
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
        "read_over_algorithmic": rd / alg,
        "dispatch_ms_under_pmc": ms_f, "launches_counted": n_f,
    }
    json.dump(rec, open(dst, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
