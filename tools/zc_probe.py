#!/usr/bin/env python3
"""Zero-copy probe (measurement tool, not product code): can kernels reading pinned host memory
over PCIe beat the H2D copy engine that bounds the host-inclusive path?

    python tools/zc_probe.py [--gib G]

On one pinned, device-mapped host buffer (fcs_host_alloc) of 1518-B frames, times
  - plain async H2D copies in 1 GiB pieces (the ceiling bench.py reports),
  - the plain read-stream kernel and the LDS-DMA stream kernel reading the host buffer directly,
  - ether_fcs_fixed_dev on the host buffer's device address (the headline kernel over PCIe),
    checked against the same kernel on a device copy,
and prints one JSON line.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=4.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import numpy as np
    import torch
    import nstack_amd as na

    lib = na.load()
    hip = ctypes.CDLL("libamdhip64.so")
    L = 1518
    n = int(a.gib * (1 << 30)) // L
    nbytes = n * L
    p = lib.fcs_host_alloc(nbytes)
    assert p, "fcs_host_alloc failed"
    d = ctypes.c_void_p()
    assert hip.hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(p), 0) == 0
    dev = torch.device("cuda:0")
    host = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
    gbuf = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(gbuf, nbytes, 0x5A, 0)
    torch.cuda.synchronize()
    host[:] = gbuf.cpu().numpy()
    sink = torch.zeros(4, dtype=torch.int32, device=dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return sorted(ts)[len(ts) // 2]

    src = torch.from_numpy(host)
    piece = 1 << 30

    def copies():
        for o in range(0, nbytes, piece):
            k = min(piece, nbytes - o)
            gbuf[o:o + k].copy_(src[o:o + k], non_blocking=True)

    res = {"bytes": nbytes, "frames": n}
    res["h2d_copy_GBs"] = round(nbytes / timed(copies) / 1e9, 2)
    res["read_stream_host_GBs"] = round(nbytes / timed(lambda: na.read_stream_dev(d.value, nbytes, sink)) / 1e9, 2)
    res["dma_stream_host_GBs"] = round(nbytes / timed(lambda: na.dma_stream_dev(d.value, nbytes, sink)) / 1e9, 2)
    out_h = torch.zeros(n, dtype=torch.int32, device=dev)
    out_d = torch.zeros(n, dtype=torch.int32, device=dev)
    res["fixed_dev_on_host_GBs"] = round(nbytes / timed(lambda: na.fixed_dev(d.value, L, L, n, out_h)) / 1e9, 2)
    copies()
    torch.cuda.synchronize()
    res["fixed_dev_on_device_GBs"] = round(nbytes / timed(lambda: na.fixed_dev(gbuf, L, L, n, out_d)) / 1e9, 2)
    res["same_crcs"] = bool(torch.equal(out_h, out_d))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
