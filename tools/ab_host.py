#!/usr/bin/env python3
"""In-process A/B of the host-inclusive entry points (measurement tool, not product code).

    python tools/ab_host.py [--gib G] [--rounds R] lib1.so lib2.so ...

Every library is a full build of the engine; all are loaded into one process and run round-robin on
the same pinned host data (bench.py's host_inclusive_1518 and host_inclusive_imix workloads):
ether_fcs_fixed_host over 1518-B frames and ether_fcs_batch_host over packed IMIX frames. Prints the
median GB/s per library and checks every library's CRCs against the first one's.
"""
import argparse
import ctypes
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    from bench import imix_lengths
    libs = []
    for p in a.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.fcs_host_alloc.restype = ctypes.c_void_p
        lib.fcs_host_alloc.argtypes = [ctypes.c_uint64]
        lib.ether_fcs_fixed_host.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                             ctypes.c_void_p]
        lib.ether_fcs_batch_host.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                             ctypes.c_void_p, ctypes.c_uint64]
        libs.append(lib)
    L = 1518
    nf = int(a.gib * (1 << 30)) // L
    ni = int(a.gib * (1 << 30) / 355.83)
    ln = imix_lengths(ni, seed=11)
    off = np.zeros(ni, dtype=np.uint64)
    np.cumsum(ln[:-1], dtype=np.uint64, out=off[1:])
    total_i = int(off[-1]) + int(ln[-1])
    size = max(nf * L, total_i)
    p = libs[0].fcs_host_alloc(size)
    buf = np.ctypeslib.as_array((ctypes.c_uint8 * size).from_address(p))
    buf[:] = np.random.default_rng(3).integers(0, 256, size, dtype=np.uint8)
    res = {}
    outs = {}
    for r in range(a.rounds + 1):
        for k, lib in enumerate(libs):
            for what in ("fixed", "imix"):
                out = np.zeros(nf if what == "fixed" else ni, dtype=np.uint32)
                t0 = time.perf_counter()
                if what == "fixed":
                    rc = lib.ether_fcs_fixed_host(p, L, L, nf, out.ctypes.data)
                    nbytes = nf * L
                else:
                    rc = lib.ether_fcs_batch_host(p, total_i, off.ctypes.data, ln.ctypes.data, out.ctypes.data, ni)
                    nbytes = total_i
                dt = time.perf_counter() - t0
                assert rc == 0, rc
                if r:
                    res.setdefault((k, what), []).append(nbytes / dt / 1e9)
                outs[(k, what)] = out
    for (k, what), v in sorted(res.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        same = bool(np.array_equal(outs[(k, what)], outs[(0, what)]))
        print(f"{what:6s} {os.path.basename(a.libs[k]):28s} median {statistics.median(v):7.2f} GB/s  "
              f"max {max(v):7.2f}  same_as_first={same}", flush=True)


if __name__ == "__main__":
    main()
