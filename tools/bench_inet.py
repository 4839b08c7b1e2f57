#!/usr/bin/env python3
"""Device-resident throughput of the Internet-checksum kernels (include/nstack_inet.h, §8f-3).

  tcp_64M_x_1480 : tcp_checksum over the TCP segment (+34, 1480 B) of 64 M x 1518-B frames
                   (the BASELINE frame population), one (src, dst) address pair per packet
  ip_64M_x_1500  : ip_checksum over the IP datagram (+14, 1500 B) of the same frames
  ip_hdr_64M_x_20: ip_checksum over the 20-B IP header only (+14): the call ip_hton makes
  imix_128M      : ip_checksum over 128 M packed packets, 7:4:1 of 64/576/1518 B (variable path)
Timing: HIP events on the launch stream around `reps` launches, after one warm-up launch.
Spot checks use the independent RFC 1071 witness of tests/golden/make_inet_golden.py (the
oracle/ restatement is reserved for tests/). Prints one JSON document.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--skip", default="")
    a = ap.parse_args()
    import numpy as np
    import torch
    import nstack_amd as na
    from make_inet_golden import witness
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(17)
    res = {"engine": na.version(), "peak_GB_s": 8000.0}

    def spot(mode, arena_t, offs, lens, addr_np, got):
        bad = 0
        for i in rng.integers(0, len(got), 48):
            o, L = int(offs[i]), int(lens[i])
            b = arena_t[o:o + L].cpu().numpy().tobytes()
            s, d = (int(addr_np[2 * i]), int(addr_np[2 * i + 1])) if addr_np is not None else (0, 0)
            bad += int(witness(mode, b, s, d) != int(got[i]))
        return bad

    n, S = a.frames, 1518
    if any(k not in a.skip for k in ("tcp", "ip")):
        frames = torch.empty(n * S + 64, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(frames, n * S + 64, 5, 0)
        addr = torch.randint(-2**31, 2**31 - 1, (2 * n,), dtype=torch.int32, device=dev)
        addr_np = addr.cpu().numpy().view(np.uint32)
        out = torch.empty(n, dtype=torch.int16, device=dev)
        idx = np.arange(n, dtype=np.int64)
        for name, mode, start, L in (("tcp_64M_x_1480", "tcp", 34, 1480), ("ip_64M_x_1500", "ip", 14, 1500),
                                     ("ip_hdr_64M_x_20", "ip", 14, 20)):
            if mode not in a.skip and name not in a.skip:
                ad = addr if mode != "ip" else None
                ms = time_dev(lambda: na.inet_fixed_dev(mode, frames.data_ptr() + start, S, L, n, ad, out,
                                                        torch.cuda.current_stream()), a.reps, torch)
                got = out.cpu().numpy().view(np.uint16)
                offs = start + idx * S
                res[name] = {"ms": ms, "packets": n, "bytes": n * L, "GB_s": n * L / ms / 1e6,
                             "frac_of_8TB_s": n * L / ms / 1e6 / 8000.0, "Mpkt_s": n / ms / 1e3,
                             "spot_bad": spot(mode, frames, offs, np.full(n, L), addr_np if ad is not None else None, got)}
                print(name, json.dumps(res[name]), flush=True)
        del frames, addr, out
        torch.cuda.empty_cache()

    if "imix" not in a.skip:
        m = 2 * n
        counts = [m * 7 // 12, m * 4 // 12]
        counts.append(m - sum(counts))
        ln_np = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), counts)
        np.random.default_rng(7).shuffle(ln_np)
        ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
        off = torch.zeros(m, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(ln[:-1].to(torch.int64), 0)
        total = int(off[-1].item()) + int(ln_np[-1])
        arena = torch.empty(total, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(arena, total, 6, 0)
        out = torch.empty(m, dtype=torch.int16, device=dev)
        ms = time_dev(lambda: na.inet_batch_dev("ip", arena, total, off, ln, None, out, m,
                                                torch.cuda.current_stream()), a.reps, torch)
        got = out.cpu().numpy().view(np.uint16)
        res["imix_128M"] = {"ms": ms, "packets": m, "bytes": total, "GB_s": total / ms / 1e6,
                            "frac_of_8TB_s": total / ms / 1e6 / 8000.0, "Mpkt_s": m / ms / 1e3,
                            "metadata_bytes": m * 12,
                            "spot_bad": spot("ip", arena, off.cpu().numpy(), ln_np, None, got)}
        print("imix_128M", json.dumps(res["imix_128M"]), flush=True)
    if "host" not in a.skip:   # host-inclusive: packets in pageable host memory, results back to host
        m = (4 << 30) // S
        host = np.random.default_rng(3).integers(0, 256, m * S + 64, dtype=np.uint8)
        off = (14 + np.arange(m, dtype=np.uint64) * S).astype(np.uint64)
        ln = np.full(m, 1500, dtype=np.uint32)
        out = np.zeros(m, dtype=np.uint16)
        na.inet_batch_host("ip", host, host.nbytes, off[:1024], ln[:1024], None, out, 1024)   # warm
        import time
        t0 = time.perf_counter()
        na.inet_batch_host("ip", host, host.nbytes, off, ln, None, out, m)
        dt = time.perf_counter() - t0
        bad = 0
        for i in rng.integers(0, m, 48):
            o = int(off[i])
            bad += int(witness("ip", host[o:o + 1500].tobytes()) != int(out[i]))
        res["host_ip_1500_pageable"] = {"packets": m, "bytes": m * 1500, "s": dt, "GB_s": m * 1500 / dt / 1e9,
                                        "Mpkt_s": m / dt / 1e6, "spot_bad": bad}
        print("host_ip_1500_pageable", json.dumps(res["host_ip_1500_pageable"]), flush=True)
    print(json.dumps(res, indent=1), flush=True)


if __name__ == "__main__":
    main()
