#!/usr/bin/env python3
"""Per-workload kernel statistics from a rocprofv3 kernel trace (measurement tool).

    python tools/kernel_stats_split.py TRACE.csv OUT.csv

rocprofv3 --stats averages every dispatch of a kernel together; bench.py launches fcs_dma_kernel
both for the 64 M x 1518 B headline (on torch's stream) and for the host-inclusive pipeline's
128 MiB chunks (the engine's own stream). This splits the statistics by (kernel, stream) so the
headline kernel's average launch time can be compared with bench.py's HIP-event timing.
"""
import collections
import csv
import statistics
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    groups = collections.OrderedDict()
    for r in csv.DictReader(open(src)):
        k = (r["Kernel_Name"], r["Stream_Id"], r["Grid_Size_X"], r["Workgroup_Size_X"])
        groups.setdefault(k, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Name", "Stream_Id", "Grid_Size_X", "Workgroup_Size_X", "Calls", "TotalDurationNs",
                    "AverageNs", "MedianNs", "MinNs", "MaxNs"])
        for (name, st, grid, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
            w.writerow([name, st, grid, wg, len(d), sum(d), round(sum(d) / len(d), 1), statistics.median(d),
                        min(d), max(d)])
    print(open(dst).read())


if __name__ == "__main__":
    main()
