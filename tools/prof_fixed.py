#!/usr/bin/env python3
"""Profiling driver: R launches of the fixed-length FCS kernel over F x L frames (HBM-resident).
Used under rocprofv3 (kernel trace / PMC passes); prints per-launch time from HIP events."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--len", type=int, default=1518)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--var", action="store_true", help="use the variable-length entry point")
    ap.add_argument("--imix", action="store_true", help="variable-length IMIX frames (7:4:1 of 64/576/1518)")
    a = ap.parse_args()
    import torch
    import nstack_amd as na
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    n, L = a.frames, a.len
    total = n * L
    if a.imix:
        import numpy as np
        a.var = True
        if n == 128 << 20:   # BASELINE configs[2] exactly as bench.py builds it (7:4:1 counts, shuffled)
            ln_np = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), [78293676, 44739242, 11184810])
            np.random.default_rng(7).shuffle(ln_np)
        else:
            ln_np = np.random.default_rng(7).choice(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.uint32), n)
        ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
        off = torch.zeros(n, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(ln[:-1].to(torch.int64), 0)
        total = int(off[-1].item()) + int(ln_np[-1])
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, total, 7, 0)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    if a.var and not a.imix:
        off = torch.arange(n, dtype=torch.int64, device=dev) * L
        ln = torch.full((n,), L, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(a.reps + 1):
        if r == 1:
            e0.record(st)
        if a.var:
            na.batch_dev(arena, total, off, ln, out, n, st)
        else:
            na.fixed_dev(arena, L, L, n, out, st)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(f"frames={n} len={L} var={a.var} imix={a.imix} ms/launch={ms:.4f} GB/s={total / ms / 1e6:.1f}")


if __name__ == "__main__":
    main()
