#!/usr/bin/env python3
"""Measure every BASELINE.json config on one MI355X (bench.py covers only the headline line).

  device-resident : 64 M x 1518 B (fixed), IMIX 128 M frames 7:4:1 of 64/576/1518 (variable,
                    seeded shuffle, packed), 16 M x 9000 B jumbo
  host-inclusive  : frames in host memory -> chunked H2D -> kernel -> D2H of CRCs, through the
                    C ABI's ether_fcs_fixed_host / ether_fcs_batch_host, for a pinned and a
                    pageable host arena
Every GPU result set is spot-checked against zlib.crc32 (stdlib CRC-32; the oracle under oracle/
is reserved for tests/ and bench.py's cpu_baseline leg). Prints one JSON document.
"""
import argparse
import ctypes
import json
import os
import sys
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def time_dev(fn, reps, torch):
    st = torch.cuda.current_stream()
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def spot_check(_, host_view_fn, crcs, idx):
    bad = 0
    for i in idx:
        b = host_view_fn(int(i))
        bad += int(zlib.crc32(b.tobytes()) != int(crcs[i]))
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--host-gib", type=float, default=8.0)
    ap.add_argument("--skip", default="")
    a = ap.parse_args()
    import numpy as np
    import torch
    import nstack_amd as na
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    o = None
    res = {"engine": na.version()}
    GIB = float(1 << 30)
    rng = np.random.default_rng(2026)

    # ---------------- fixed 64 M x 1518 ----------------
    if "fixed" not in a.skip:
        n, L = 64 << 20, 1518
        arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(arena, n * L, 1, 0)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ms = time_dev(lambda: na.fixed_dev(arena, L, L, n, out, torch.cuda.current_stream()), a.reps, torch)
        crcs = out.cpu().numpy().view(np.uint32)
        idx = rng.integers(0, n, 64)
        bad = spot_check(o, lambda i: arena[i * L:(i + 1) * L].cpu().numpy(), crcs, idx)
        res["fixed_64M_x_1518"] = {"ms": ms, "GiB_s": n * L / ms / 1e-3 / GIB, "GB_s": n * L / ms / 1e6,
                                   "Mframes_s": n / ms / 1e3, "spot_bad": bad}
        # RX verify mode over the same frames (random trailers: essentially every frame fails,
        # the worst case for the bad-frame counter)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        nbad = torch.zeros(1, dtype=torch.int64, device=dev)
        ms_v = time_dev(lambda: na.verify_fixed_dev(arena, L, L, n, ok, nbad, torch.cuda.current_stream()),
                        a.reps, torch)
        res["verify_fixed_64M_x_1518"] = {"ms": ms_v, "GB_s": n * L / ms_v / 1e6, "bad": int(nbad.item()),
                                          "expected_bad": int((torch.from_numpy(crcs.view(np.int32)) !=
                                                               0x2144DF1C).sum())}
        del arena, out, ok
        torch.cuda.empty_cache()

    # ---------------- IMIX 128 M frames ----------------
    if "imix" not in a.skip:
        n = 128 << 20
        counts = [78293676, 44739242, 11184810]
        ln_np = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), counts)
        np.random.default_rng(7).shuffle(ln_np)
        ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
        off = torch.zeros(n, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(ln[:-1].to(torch.int64), 0)
        total = int(off[-1].item()) + int(ln_np[-1])
        arena = torch.empty(total, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(arena, total, 2, 0)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ms = time_dev(lambda: na.batch_dev(arena, total, off, ln, out, n, torch.cuda.current_stream()), a.reps, torch)
        crcs = out.cpu().numpy().view(np.uint32)
        offs = off.cpu().numpy()
        idx = rng.integers(0, n, 64)
        bad = spot_check(o, lambda i: arena[int(offs[i]):int(offs[i]) + int(ln_np[i])].cpu().numpy(), crcs, idx)
        res["imix_128M"] = {"ms": ms, "bytes": total, "GiB_s": total / ms / 1e-3 / GIB, "GB_s": total / ms / 1e6,
                            "Mframes_s": n / ms / 1e3, "avg_len": total / n, "spot_bad": bad,
                            "metadata_bytes": n * 12}
        del arena, out, off, ln
        torch.cuda.empty_cache()

    # ---------------- jumbo 16 M x 9000 ----------------
    if "jumbo" not in a.skip:
        n, L = 16 << 20, 9000
        arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(arena, n * L, 3, 0)
        out = torch.empty(n, dtype=torch.int32, device=dev)
        ms = time_dev(lambda: na.fixed_dev(arena, L, L, n, out, torch.cuda.current_stream()), a.reps, torch)
        crcs = out.cpu().numpy().view(np.uint32)
        idx = rng.integers(0, n, 64)
        bad = spot_check(o, lambda i: arena[i * L:(i + 1) * L].cpu().numpy(), crcs, idx)
        res["jumbo_16M_x_9000"] = {"ms": ms, "GiB_s": n * L / ms / 1e-3 / GIB, "GB_s": n * L / ms / 1e6,
                                   "Mframes_s": n / ms / 1e3, "spot_bad": bad}
        del arena, out
        torch.cuda.empty_cache()

    # ---------------- host-inclusive ----------------
    if "host" not in a.skip:
        L = 1518
        n = int(a.host_gib * GIB) // L
        nbytes = n * L
        lib = na.load()
        p = lib.fcs_host_alloc(nbytes)
        assert p, "pinned alloc failed"
        pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(d, nbytes, 4, 0)
        torch.cuda.synchronize()
        pinned[:] = d.cpu().numpy()
        del d
        torch.cuda.empty_cache()
        out = np.zeros(n, dtype=np.uint32)
        na.fixed_host(p, L, L, min(n, 1 << 16), out)   # warm the pipeline buffers
        t0 = time.perf_counter()
        na.fixed_host(p, L, L, n, out)
        t1 = time.perf_counter()
        idx = rng.integers(0, n, 64)
        bad = spot_check(o, lambda i: pinned[i * L:(i + 1) * L], out, idx)
        res["host_fixed_pinned"] = {"frames": n, "bytes": nbytes, "s": t1 - t0,
                                    "GiB_s": nbytes / (t1 - t0) / GIB, "GB_s": nbytes / (t1 - t0) / 1e9,
                                    "spot_bad": bad}
        pageable = np.array(pinned)          # ordinary (pageable) host memory
        out2 = np.zeros(n, dtype=np.uint32)
        t0 = time.perf_counter()
        na.fixed_host(pageable, L, L, n, out2)
        t1 = time.perf_counter()
        res["host_fixed_pageable"] = {"frames": n, "bytes": nbytes, "s": t1 - t0,
                                      "GiB_s": nbytes / (t1 - t0) / GIB, "GB_s": nbytes / (t1 - t0) / 1e9,
                                      "same_as_pinned": bool(np.array_equal(out, out2))}
        # IMIX from host memory (pinned arena)
        m = 0
        lens = []
        while True:
            x = [64] * 7 + [576] * 4 + [1518]
            if m + sum(x) > nbytes:
                break
            lens += x
            m += sum(x)
        ln_np = np.array(lens, dtype=np.uint32)
        np.random.default_rng(9).shuffle(ln_np)
        off_np = np.zeros(len(ln_np), dtype=np.uint64)
        off_np[1:] = np.cumsum(ln_np[:-1], dtype=np.uint64)
        out3 = np.zeros(len(ln_np), dtype=np.uint32)
        t0 = time.perf_counter()
        na.batch_host(p, nbytes, off_np, ln_np, out3, len(ln_np))
        t1 = time.perf_counter()
        res["host_imix_pinned"] = {"frames": len(ln_np), "bytes": m, "s": t1 - t0,
                                   "GiB_s": m / (t1 - t0) / GIB, "GB_s": m / (t1 - t0) / 1e9,
                                   "Mframes_s": len(ln_np) / (t1 - t0) / 1e6,
                                   "spot_bad": spot_check(o, lambda i: pinned[int(off_np[i]):int(off_np[i]) + int(ln_np[i])],
                                                          out3, rng.integers(0, len(ln_np), 64))}
        lib.fcs_host_free(p)

    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
