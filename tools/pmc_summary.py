#!/usr/bin/env python3
"""Summarise tools/pmc.sh output: per-dispatch average of every counter for the FCS kernel."""
import collections
import csv
import glob
import json
import os
import sys


def summarize(outdir, kernel="fcs_kernel"):
    res = {}
    for p in sorted(glob.glob(os.path.join(outdir, "p*", "run_counter_collection.csv"))):
        rows = list(csv.DictReader(open(p)))
        agg = collections.defaultdict(float)
        disp = set()
        for r in rows:
            if kernel not in r["Kernel_Name"]:
                continue
            disp.add(r["Dispatch_Id"])
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
        for k, v in agg.items():
            res[k] = v / max(1, len(disp))
    times = []
    for p in sorted(glob.glob(os.path.join(outdir, "p*", "run_kernel_trace.csv"))):
        for r in csv.DictReader(open(p)):
            if kernel in r["Kernel_Name"]:
                times.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    res["kernel_ms_profiled_mean"] = sum(times) / len(times) if times else None
    return res


if __name__ == "__main__":
    r = summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "fcs_kernel")
    print(json.dumps(r, indent=1))
