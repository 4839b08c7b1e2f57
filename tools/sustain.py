#!/usr/bin/env python3
"""Sustained-load curve: per-launch device time of N back-to-back FCS launches (measurement tool).

    [NSTACK_FCS_LIB=...] python tools/sustain.py [--launches N] [--frames F] [--len L]

HIP events are recorded between consecutive launches on one stream, so the GPU never idles; the
printed series shows how the clock (power limiter) settles under continuous load.
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--launches", type=int, default=150)
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--len", type=int, default=1518)
    a = ap.parse_args()
    import torch
    import nstack_amd as na
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    n, L = a.frames, a.len
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, 5, 0)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.launches + 1)]
    ev[0].record(st)
    for i in range(a.launches):
        na.fixed_dev(arena, L, L, n, out, st)
        ev[i + 1].record(st)
    torch.cuda.synchronize()
    ms = [ev[i].elapsed_time(ev[i + 1]) for i in range(a.launches)]
    gbs = [n * L / (m * 1e-3) / 1e9 for m in ms]
    chunks = [sum(gbs[i:i + 10]) / len(gbs[i:i + 10]) for i in range(0, len(gbs), 10)]
    print(json.dumps({"lib": os.path.basename(na.LIB_PATH), "first_ms": round(ms[0], 3),
                      "GBs_per_10_launches": [round(x) for x in chunks],
                      "last50_GBs": round(sum(gbs[-50:]) / 50)}))


if __name__ == "__main__":
    main()
