#!/usr/bin/env python3
"""One-process A/B of the Internet-checksum kernels (measurement tool): the LDS-DMA kernels
(inet_csum_set_dma_threshold(0)) against the flat chunk stream (dma threshold at infinity),
alternating, HIP events on the launch stream, median of R. Fixed strides (IP datagrams and TCP
segments of 1518-B frames), then variable batches: IMIX packed (7:4:1 of 64/576/1518, shuffled)
and the same lengths one per 1536-B slot (not packed: the stream kernel's flat windows).

    python tools/inet_ab.py [--frames N] [--imix-frames M] [--rounds R]
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
    ap.add_argument("--imix-frames", type=int, default=128 << 20)
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
    del buf, addr, outs
    torch.cuda.empty_cache()
    # variable batches
    import numpy as np
    m = a.imix_frames
    rng = np.random.default_rng(7)
    lens = rng.permutation(np.tile(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.int64), (m + 11) // 12)[:m])
    cases = [("imix packed", lens, np.concatenate([[0], np.cumsum(lens)[:-1]]), int(lens.sum())),
             ("imix slots", lens, np.arange(m, dtype=np.int64) * 1536, m * 1536),
             ("hdr 20 B", np.full(m, 20, dtype=np.int64), 14 + np.arange(m, dtype=np.int64) * 1518, m * 1518)]
    for name, lens, offs, span in cases:
        if span > (200 << 30):
            continue
        arena = torch.empty(span + 64, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(arena, arena.numel(), 0x1E8, 0)
        d_off = torch.from_numpy(offs.astype(np.int64)).to(dev)
        d_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        o2 = {k: torch.empty(m, dtype=torch.int16, device=dev) for k in ("dma", "flat")}
        t = {"dma": [], "flat": []}
        for r in range(a.rounds + 1):
            for k in ("dma", "flat"):
                na.inet_set_dma_threshold(0 if k == "dma" else (1 << 63))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                na.inet_batch_dev("ip", arena, span + 64, d_off, d_len, None, o2[k], m)
                e1.record(st)
                torch.cuda.synchronize()
                if r:
                    t[k].append(e0.elapsed_time(e1))
        same = torch.equal(o2["dma"], o2["flat"])
        for k in ("dma", "flat"):
            ms = statistics.median(t[k])
            print(f"inet {name:11s} {k:5s} median {ms:8.3f} ms  {int(lens.sum()) / ms / 1e6:8.1f} GB/s  same={same}",
                  flush=True)
        del arena, d_off, d_len, o2
        torch.cuda.empty_cache()
    na.inet_set_dma_threshold(16384)


if __name__ == "__main__":
    main()
