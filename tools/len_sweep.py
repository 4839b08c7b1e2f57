#!/usr/bin/env python3
"""Fixed-length rate sweep (measurement tool): ether_fcs_fixed_dev over about 24 GiB of packed
frames per length, device-resident, HIP events on the launch stream, median of R launches after one
untimed launch. One JSON line per length: the rate and which kernel family the host picks for it
(fcs_launch.hpp / fcs_engine.cpp selection, restated here for the report only).

    python tools/len_sweep.py [--lens 64,128,...] [--gib 24] [--reps 5]
"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

DEFAULT_LENS = [64, 128, 256, 512, 576, 768, 869, 870, 1000, 1156, 1157, 1250, 1350, 1476, 1477, 1490, 1500, 1514, 1518,
                1524, 1525, 1536, 1600, 1787, 1900, 1988, 2500, 3000, 4096, 6000, 9000, 9216, 16384, 65536]


def family(L):
    """The kernel family a large packed batch of L-byte frames takes (as selected in the library)."""
    if L <= 128:
        return "short (lane per frame)"
    if 130 <= L <= 399:
        return "wide, 4 lanes (flat if bank-phased)"
    if 400 <= L <= 868:
        return "wide, 8 lanes (flat if bank-phased)"
    if 870 <= L <= 1476:
        return "wide (mid, 6 KiB slots)"
    if L <= 869:
        return "flat"
    if L <= 1495:
        return "wide WD26"
    if L <= 1524:
        return "lds-dma (headline)"
    if L <= 1604:
        return "wide WD26"
    if L <= 1787:
        return "wide WD30"
    if L <= 1988:
        return "wide WD32"
    m = (L + 1523) // 1524
    order = [24, 15, 16, 18, 19, 20, 22, 23, 26, 30, 32]   # fcs_launch.hpp segment_wd's candidates
    cover = {w: 15 * (4 * w - 4) + 4 * w for w in order}
    cover[24] = 1524
    costs = [-(-L // cover[w]) * (w + 8) for w in order]
    wd = order[costs.index(min(costs))]
    if m >= 4 or (m == 3 and (L > 3072 or wd != 24)) or (m == 2 and L >= 1950):
        return "segment (interleaved)" if wd == 24 else f"segment (interleaved, WD{wd})"
    return "generic"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", nargs="+", default=[",".join(map(str, DEFAULT_LENS))],
                    help="lengths, comma- or space-separated")
    ap.add_argument("--gib", type=float, default=24.0)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    import nstack_amd as na
    na.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    cap = int(a.gib * (1 << 30))
    arena = torch.empty(cap + 64, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, cap + 64, 5, 0)
    st = torch.cuda.current_stream()
    for L in [int(x) for x in ",".join(a.lens).split(",") if x]:
        n = cap // L
        out = torch.empty(n, dtype=torch.int32, device=dev)
        na.fixed_dev(arena, L, L, n, out, st)   # untimed
        times = []
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            na.fixed_dev(arena, L, L, n, out, st)
            e1.record(st)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        ms = statistics.median(times)
        print(json.dumps({"len": L, "frames": n, "bytes": n * L, "ms": round(ms, 4),
                          "GB_s": round(n * L / ms / 1e6, 1), "frac_of_8TBs": round(n * L / ms / 1e6 / 8000, 4),
                          "Mframes_s": round(n / ms / 1e3, 1), "kernel": family(L),
                          "route": na.fixed_route(arena.data_ptr(), L, L, n)}), flush=True)
        del out


if __name__ == "__main__":
    main()
