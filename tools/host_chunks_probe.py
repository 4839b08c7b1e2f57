#!/usr/bin/env python3
"""Probe of ether_fcs_batch_host over several pipeline chunks (measurement/debug tool): each layout
of tests/test_gpu_parity.py::test_batch_host_many_chunks, timed stage by stage, flushed per line."""
import faulthandler
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def imix(n, seed):
    counts = [n * 7 // 12, n * 4 // 12]
    counts.append(n - sum(counts))
    ln = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), counts)
    np.random.default_rng(seed).shuffle(ln)
    return ln


def main():
    faulthandler.dump_traceback_later(60, repeat=True)
    import zlib
    import nstack_amd as na
    na.load()
    for layout in sys.argv[1:] or ["packed", "gapped", "shuffled", "jumbo_mix"]:
        t0 = time.time()
        rng = np.random.default_rng(["packed", "gapped", "shuffled", "jumbo_mix"].index(layout) + 40)
        n = 1_200_000
        ln = imix(n, 17).astype(np.uint64)
        if layout == "jumbo_mix":
            ln[rng.integers(0, n, 3000)] = 9000
            ln[rng.integers(0, n, 3000)] = 0
        gap = rng.integers(0, 600, n).astype(np.uint64) if layout == "gapped" else np.zeros(n, dtype=np.uint64)
        start = np.zeros(n, dtype=np.uint64)
        start[1:] = np.cumsum(ln[:-1] + gap[:-1], dtype=np.uint64)
        off = start.copy()
        if layout == "shuffled":
            perm = rng.permutation(n)
            off = start[perm]
            ln = ln[perm]
        total = int((off + ln).max()) + 16
        arena = rng.integers(0, 256, total, dtype=np.uint8)
        out = np.zeros(n, dtype=np.uint32)
        print(f"{layout}: data {time.time() - t0:.2f} s", flush=True)
        t1 = time.time()
        na.batch_host(arena, arena.nbytes, off, ln.astype(np.uint32), out, n)
        print(f"{layout}: batch_host {time.time() - t1:.3f} s ({total / (time.time() - t1) / 1e9:.1f} GB/s of span)", flush=True)
        idx = rng.integers(0, n, 2000)
        bad = sum(int(zlib.crc32(arena[int(off[i]):int(off[i]) + int(ln[i])].tobytes()) != int(out[i])) for i in idx)
        print(f"{layout}: sampled 2000, bad {bad}", flush=True)


if __name__ == "__main__":
    main()
