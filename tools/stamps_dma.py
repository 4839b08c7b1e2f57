#!/usr/bin/env python3
"""Per-wave s_memtime stamps of an FCS_STAMPS build of fcs_dma_kernel or fcs_segil_kernel (--len over
1524 B, e.g. 9000; measurement tool): cycles per
item spent waiting for the slot DMA (vmcnt at the loop top) vs. the whole item, and the in-kernel
shader clock (s_memtime / s_memrealtime at 100 MHz, MI355X_MICROARCH.md DVFS item 6).

    NSTACK_FCS_LIB=tools/variants/libfcs_stamps.so python tools/stamps_dma.py [--frames F]
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--len", type=int, default=1518)
    ap.add_argument("--reps", type=int, default=6)
    a = ap.parse_args()
    import torch
    import nstack_amd as na
    lib = na.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    n, L = a.frames, a.len
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, 11, 0)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    dbg = torch.zeros(256 * 16 * 8, dtype=torch.int64, device=dev)   # up to 16 waves per CU
    st = torch.cuda.current_stream()
    lib.fcs_debug_set_sink.argtypes = [ctypes.c_void_p]
    lib.fcs_debug_set_sink(dbg.data_ptr())
    for r in range(a.reps):   # warm, back-to-back launches; the last one's stamps are reported
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        na.fixed_dev(arena, L, L, n, out, st)
        e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    d = dbg.view(-1, 8).cpu()
    live = d[:, 2] > 0
    d = d[live]
    items = int(d[:, 2].sum())
    wait = float(d[:, 0].sum()) / items
    allc = float(d[:, 1].sum()) / items
    clk = float((d[:, 4].double() / d[:, 3].double()).median()) * 0.1   # GHz
    print(f"ms {ms:.3f}  GB/s {n * L / ms / 1e6:.1f}  waves {int(live.sum())}  items/wave {items / int(live.sum()):.1f}")
    print(f"cycles per item: total {allc:.0f}  waiting for the slot DMA {wait:.0f} ({100 * wait / allc:.1f} %)")
    rt_ms = float(d[:, 3].double().median()) / 1e5
    t0 = int(d[:, 5].min())
    st = (d[:, 5] - t0).double() / 1e5
    en = (d[:, 6] - t0).double() / 1e5
    q = torch.tensor([0.0, 0.1, 0.5, 0.9, 1.0], dtype=torch.float64)
    print("wave start ms (min/10/50/90/max):", [round(float(x), 3) for x in torch.quantile(st, q)])
    print("wave end   ms (min/10/50/90/max):", [round(float(x), 3) for x in torch.quantile(en, q)])
    xcc = d[:, 7] & 7
    for x in range(8):
        sel = xcc == x
        if int(sel.sum()):
            print(f"  XCC {x}: waves {int(sel.sum())}  end median {float(en[sel].median()):.3f} ms  max {float(en[sel].max()):.3f}")
    print(f"in-kernel shader clock {clk:.3f} GHz; loop wall time per wave (s_memrealtime, 100 MHz) {rt_ms:.3f} ms")
    # what decides the end: the spread of the waves' finishing times against the kernel's span,
    # per XCD, and the last waves' share of items
    span = float(en.max())
    med = float(en.median())
    print(f"tail: last wave ends {span - med:.3f} ms after the median wave ({100 * (span - med) / span:.2f} % of the span);"
          f" items per wave min/median/max {int(d[:, 2].min())}/{int(d[:, 2].median())}/{int(d[:, 2].max())}")
    per_x = [float(en[xcc == x].median()) for x in range(8) if int((xcc == x).sum())]
    if per_x:
        print(f"XCD median end spread {max(per_x) - min(per_x):.3f} ms ({100 * (max(per_x) - min(per_x)) / span:.2f} %)")


if __name__ == "__main__":
    main()
