#!/usr/bin/env python3
"""Write profiles/<round>_pmc_traffic*.json from separate rocprofv3 FETCH_SIZE / WRITE_SIZE passes.

    python tools/traffic_summary.py SRC DST [--kernel K] [--frames F] [--len L|imix] [--alg BYTES]
                                    [--meta BYTES] [--sub-fetch pmc_fetch] [--sub-write pmc_write]

HBM bytes per launch of one kernel at one workload, corrected as MI355X_MICROARCH.md's HBM section
prescribes: FETCH_SIZE (KB) x 2 on gfx950 for wide streaming reads (16 B per lane, global_load and
LDS-DMA alike), WRITE_SIZE (KB) as is, KB = 1024 B. bench.py reads the newest matching file for
roofline.traffic (kernel name, frames and len must match its workload).
"""
import argparse
import csv
import glob
import json
import os


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
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("dst")
    ap.add_argument("--kernel", default="fcs_dma_kernel")
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--len", default="1518")
    ap.add_argument("--alg", type=int, default=None, help="algorithmic bytes per launch (default frames x len)")
    ap.add_argument("--meta", type=int, default=0, help="metadata bytes per launch (offsets, lengths, CRCs)")
    ap.add_argument("--sub-fetch", default="pmc_fetch")
    ap.add_argument("--sub-write", default="pmc_write")
    ap.add_argument("--command", default="tools/profile_round.sh")
    a = ap.parse_args()
    L = int(a.len) if a.len.isdigit() else a.len
    alg = a.alg if a.alg is not None else a.frames * int(L)
    fetch, n_f, ms_f = per_dispatch(os.path.join(a.src, a.sub_fetch), "FETCH_SIZE", a.kernel)
    write, n_w, ms_w = per_dispatch(os.path.join(a.src, a.sub_write), "WRITE_SIZE", a.kernel)
    rd = fetch * 1024 * 2
    wr = write * 1024
    rec = {
        "round": int(os.path.basename(a.dst)[1:3]),
        "kernel": "fcs::" + a.kernel,
        "frames": a.frames, "len": L, "algorithmic_bytes_per_launch": alg, "metadata_bytes_per_launch": a.meta,
        "command": a.command,
        "FETCH_SIZE_kb_per_launch": fetch, "WRITE_SIZE_kb_per_launch": write,
        "correction": "MI355X_MICROARCH.md HBM: on gfx950 FETCH_SIZE reports 1/2 of the bytes of a wide "
                      "coalesced read -> x2; WRITE_SIZE taken as is; KB = 1024 B",
        "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
        "read_over_algorithmic": rd / alg,
        "read_over_algorithmic_plus_metadata": rd / (alg + a.meta),
        "dispatch_ms_under_pmc": ms_f, "launches_counted": n_f,
    }
    json.dump(rec, open(a.dst, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
