#!/usr/bin/env python3
"""One-process A/B of the Internet-checksum kernels on fixed-stride batches (measurement tool):
the LDS-DMA kernel (inet_csum_set_dma_threshold(0)) against the flat chunk stream
(dma threshold at infinity), alternating, HIP events on the launch stream, median of R.

    python tools/inet_ab.py [--frames N] [--rounds R]
"""
import argparse
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--rounds", type=int, default=8)
    a = ap.parse_args()
    import torch
    import nstack_amd as na
    na.load()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    n, stride = a.frames, 1518
    buf = torch.empty(n * stride + 64, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(buf, buf.numel(), 0x1E7, 0)
    addr = torch.randint(-2**31, 2**31 - 1, (2 * n,), dtype=torch.int32, device=dev)
    outs = {k: torch.empty(n, dtype=torch.int16, device=dev) for k in ("dma", "flat")}
    st = torch.cuda.current_stream()
    for mode, start, L in (("ip", 14, 1500), ("tcp", 34, 1480)):
        t = {"dma": [], "flat": []}
        for r in range(a.rounds + 1):
            for k in ("dma", "flat"):
                na.inet_set_dma_threshold(0 if k == "dma" else (1 << 63))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                na.inet_fixed_dev(mode, buf.data_ptr() + start, stride, L, n, None if mode == "ip" else addr, outs[k])
                e1.record(st)
                torch.cuda.synchronize()
                if r:
                    t[k].append(e0.elapsed_time(e1))
        same = torch.equal(outs["dma"], outs["flat"])
        for k in ("dma", "flat"):
            ms = statistics.median(t[k])
            print(f"inet {mode:3s} {k:5s} median {ms:8.3f} ms  {n * L / ms / 1e6:8.1f} GB/s  "
                  f"span {n * stride / ms / 1e6:8.1f} GB/s  same={same}", flush=True)
    na.inet_set_dma_threshold(16384)


if __name__ == "__main__":
    main()
