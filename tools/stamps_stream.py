#!/usr/bin/env python3
"""Per-wave s_memtime phase sums of an FCS_STAMPS build of fcs_stream_kernel (measurement tool):
cycles per item in the marks, the slot wait, the words + next DMA + chain, and the rest
(contributions, closes); cycles per unit prologue (metadata loads, packed check, first DMA).

    NSTACK_FCS_LIB=tools/variants/libfcs_ststamps.so python tools/stamps_stream.py [--frames F]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=128 << 20)
    ap.add_argument("--reps", type=int, default=4)
    a = ap.parse_args()
    import numpy as np
    import torch
    import nstack_amd as na
    from bench import imix_lengths
    lib = na.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    n = a.frames
    ln_np = imix_lengths(n)
    ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
    off = torch.zeros(n, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(ln[:-1].to(torch.int64), 0)
    total = int(off[-1].item()) + int(ln_np[-1])
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, total, 11, 0)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(256 * 16 * 8, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    lib.fcs_debug_set_sink.argtypes = [ctypes.c_void_p]
    lib.fcs_debug_set_sink(dbg.data_ptr())
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        na.batch_dev(arena, total, off, ln, out, n, st)
        e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    d = dbg.view(-1, 8).cpu().double()
    live = d[:, 5] > 0
    d = d[live]
    items, units = float(d[:, 5].sum()), float(d[:, 6].sum())
    names = ["unit prologue (per unit)", "marks", "slot wait", "words+DMA+chain", "rest"]
    print(f"ms {ms:.3f}  GB/s {total / ms / 1e6:.1f}  waves {int(live.sum())}  items/wave {items / int(live.sum()):.1f}  "
          f"items/unit {items / units:.1f}")
    tot = float(d[:, 7].sum())
    print(f"cycles per item (all): {tot / items:.0f}")
    print(f"  {names[0]}: {float(d[:, 0].sum()) / units:.0f} per unit = {float(d[:, 0].sum()) / items:.0f} per item")
    for i in range(1, 5):
        print(f"  {names[i]}: {float(d[:, i].sum()) / items:.0f}")
    acc = float(d[:, :5].sum())
    print(f"  unaccounted (unit closes, dispenser): {(tot - acc) / items:.0f}")
    # every wave runs from about the kernel's start to its end, so a wave's whole s_memtime count
    # over the launch time is the in-kernel shader clock (an upper bound on the wave's span)
    print(f"in-kernel shader clock ~{float(d[:, 7].median()) / (ms * 1e-3) / 1e9:.3f} GHz "
          f"(median wave cycles {float(d[:, 7].median()):.0f} over {ms:.3f} ms)")


if __name__ == "__main__":
    main()
