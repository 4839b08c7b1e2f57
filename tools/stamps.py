#!/usr/bin/env python3
"""Per-wave s_memtime stamps from an FCS_STAMPS build of the single-segment kernel (measurement
tool). Reports mean shader-clock cycles per item for the CRC chain and for the whole item
(chain + merge + lane shift + reduce + store), and the kernel's cycles per item per wave.

    NSTACK_FCS_LIB=tools/variants/libfcs_stamps.so python tools/stamps.py [--frames F]
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
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    dbg = torch.zeros(cus * 16 * 4, dtype=torch.int64, device=dev)
    st = torch.cuda.current_stream()
    lib.fcs_debug_set_sink.argtypes = [ctypes.c_void_p]
    lib.fcs_debug_set_sink(dbg.data_ptr())
    na.fixed_dev(arena, L, L, n, out, st)          # warm
    torch.cuda.synchronize()
    dbg.zero_()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    na.fixed_dev(arena, L, L, n, out, st)
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    d = dbg.view(-1, 4).cpu()
    items = int(d[:, 2].sum())
    chain = float(d[:, 0].sum()) / items
    proc = float(d[:, 1].sum()) / items
    waves = int((d[:, 2] > 0).sum())
    per_wave_items = items / waves
    # s_memtime counts the shader clock (SCLK) on CDNA: derive the mean clock from the stamps
    print(f"ms {ms:.3f}  GB/s {n * L / ms / 1e6:.1f}  waves {waves}  items/wave {per_wave_items:.1f}")
    print(f"cycles per item: chain {chain:.0f}  process {proc:.0f}")
    print(f"kernel ms per item per wave {ms / per_wave_items * 1e3:.3f} us")


if __name__ == "__main__":
    main()
