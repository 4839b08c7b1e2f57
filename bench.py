#!/usr/bin/env python3
"""bench.py — device-resident CRC-32 FCS throughput on 1518-B frames (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--frames-per-gpu F] [--len L]

--gpus N is authoritative: started without a launcher (no WORLD_SIZE), bench.py starts the N ranks
itself under torch.distributed.run before any GPU call; under a launcher WORLD_SIZE must equal N
(else exit 1). config.devices lists every rank's HIP device and PCI address.

A "step" is ONE launch of the FCS kernel over one batch: F (default 64 M) x 1518-B frames per
GPU, already resident in HBM (BASELINE configs[1]; configs[4] = the same per GPU at N = 8).
For N > 1 one process runs per GPU (torch.distributed.run, by the driver or by bench.py); frames shard
embarrassingly (each rank owns a contiguous slice of the global frame stream), so the only
collectives are the timing barrier and the max-over-ranks of the elapsed time — none on the
data path. value = bytes of all ranks / max rank time, in GiB/s.

Printed (rank 0, one JSON line): the contract fields plus
  roofline     — the FCS kernel's achieved algorithmic GB/s (frame bytes per launch / average
                 launch time from HIP events on the launch stream) against the 8 TB/s HBM peak;
                 `traffic` = HBM bytes per launch from the committed rocprofv3 PMC summary
                 (profiles/*pmc_traffic*.json), or null; read_stream_gbs = a pure read kernel over
                 the same buffer (plain 16-B loads), dma_stream_gbs = the kernel's own LDS-DMA loads
                 and schedule without the CRC work (the measured read ceilings);
  cpu_baseline — the reference's own src/ether_fcs.c (oracle/_ref, its Makefile flags) timed on
                 1 M x 1518 B on one host thread, the oracle port beside it; rank 0, N = 1;
  configs      — (N = 1) the other single-GPU BASELINE configs, each timed in this process after the
                 headline and freed before the next: imix_128M (configs[2]), jumbo_16M_x_9000
                 (configs[3]; IMIX also beside its kernel's own load ceiling, stream_load_gbs = the
                 arena-stream kernel's units, items and slot DMA without the CRC work) and
                 host_inclusive_1518 (frames in pinned host memory -> H2D -> kernel
                 -> D2H, PCIe-bound; never `value`; its ceiling h2d_copy_gbs = plain async copies of
                 the same pinned arena), each with ms, GB/s, roofline frac (the HBM-bound ones also
                 against the headline run's two measured read ceilings) and a zlib spot check of
                 sampled frames.
For N > 1 the timing barrier and the max-over-ranks use gloo on the host: no RCCL collective
anywhere (BASELINE north_star), and nothing but 8 bytes of timing crosses ranks.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "device-resident CRC-32 FCS GiB/s on 1518-B frames, 1/2/4/8 MI355X; % HBM peak"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
GIB = float(1 << 30)
SEED = 0x4E535441434B        # "NSTACK"


def shard_range(total_frames: int, world: int, rank: int, lengths=None):
    """Contiguous frame range of `rank` (BASELINE configs[4]: 512 M frames over 8 GPUs), from the
    engine's own shard planner (fcs_shard_plan; byte-balanced when `lengths` is given)."""
    import nstack_amd as na
    cut = na.shard_plan(total_frames, world, lengths)
    return cut[rank], cut[rank + 1]


def aggregate(bytes_per_rank, times):
    """Whole-job throughput: all ranks' bytes over the slowest rank's time."""
    t = max(times)
    return sum(bytes_per_rank) / t, t


def splitmix_bytes(seed: int, byte_off: int, n: int):
    """Host copy of the device generator (fcs_fill_splitmix64_dev): 8-byte word q of the stream is
    splitmix64(seed + q), little-endian. Used to re-create sampled frames for the spot check."""
    import numpy as np
    q0, q1 = byte_off >> 3, (byte_off + n + 7) >> 3
    with np.errstate(over="ignore"):
        x = np.arange(q0, q1, dtype=np.uint64) + np.uint64(seed & (2**64 - 1))
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
    b = x.astype("<u8").view(np.uint8)
    s = byte_off - 8 * q0
    return b[s:s + n]


def _traffic_key(p):
    """Sort key of a PMC summary: round, then a round's first bundle (profiles/rNN_pmc_traffic*.json)
    before its tagged re-runs (profiles/rNN_<tag>/rNN_<tag>_pmc_traffic*.json), as _profile_bundles."""
    import re
    m = re.match(r"r(\d+)(?:_([a-z0-9]+))?_pmc_traffic", os.path.basename(p))
    tagged = m is not None and m.group(2) is not None and os.path.dirname(p) != os.path.join(ROOT, "profiles")
    return (int(m.group(1)) if m else -1, 1 if tagged else 0, m.group(2) or "" if m else "", os.path.basename(p))


def _load_pmc_traffic(frames: int, L, kernel: str = None):
    """HBM bytes per launch from the newest committed rocprofv3 PMC summary of this workload
    (profiles/rNN_pmc_traffic*.json and tagged bundles under profiles/rNN_<tag>/; later rounds and
    later bundles of a round sort later), if one matches."""
    best = None
    paths = glob.glob(os.path.join(ROOT, "profiles", "**", "*pmc_traffic*.json"), recursive=True)
    for p in sorted(paths, key=_traffic_key):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if kernel is not None and kernel not in d.get("kernel", ""):
            continue
        if d.get("frames") == frames and d.get("len") == L and d.get("hbm_bytes_per_launch"):
            best = (d["hbm_bytes_per_launch"], os.path.relpath(p, ROOT))
    return best


def _profile_bundles():
    """Committed kernel-statistics files of this command (tools/kernel_stats_split.py), oldest first:
    profiles/rNN_bench_kernel_stats_split.csv (a round's first bundle), then any later bundle of the
    same round (profiles/rNN_<tag>/rNN_<tag>_bench_kernel_stats_split.csv, e.g. r03_final)."""
    import re
    out = []
    for p in glob.glob(os.path.join(ROOT, "profiles", "**", "r*_bench_kernel_stats_split.csv"), recursive=True):
        m = re.match(r"r(\d+)(?:_([a-z0-9]+))?_bench_kernel_stats_split\.csv$", os.path.basename(p))
        if m:   # a round's first bundle sorts before its tagged re-runs; tags in commit order by mtime-free name
            out.append(((int(m.group(1)), 0 if m.group(2) is None else 1, m.group(2) or ""), p))
    return [p for _, p in sorted(out)]


def _load_kernel_profile(kernel: str, nbytes: int):
    """The committed rocprofv3 kernel statistics of this command: the `kernel` row carrying the most
    time (the headline launches; the host-inclusive pipeline launches the same kernel on small chunks)
    of the NEWEST bundle (not the faster of two), with every bundle of that round listed
    beside it. Returns the traced average ms per launch and the roofline fraction it gives, beside the
    in-run HIP-event one."""
    import csv
    files = _profile_bundles()

    def row(path):
        best = None
        for r in csv.DictReader(open(path)):
            if r["Name"].startswith(kernel) and (best is None or int(r["TotalDurationNs"]) > int(best["TotalDurationNs"])):
                best = r
        return best
    rows = [(p, row(p)) for p in files]
    rows = [(p, r) for p, r in rows if r is not None]
    if not rows:
        return None
    path, best = rows[-1]
    ms = float(best["AverageNs"]) / 1e6
    rnd = os.path.basename(path)[:3]
    return {"profile_kernel_ms": round(ms, 4), "profile_median_ms": round(float(best["MedianNs"]) / 1e6, 4),
            "profile_calls": int(best["Calls"]), "profile_frac": round(nbytes / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "profile_source": os.path.relpath(path, ROOT),
            "profile_bundles_this_round": {os.path.relpath(p, ROOT): round(float(r["AverageNs"]) / 1e6, 4)
                                           for p, r in rows if os.path.basename(p).startswith(rnd)}}


def _time_launches(fn, reps, stream, torch):
    """Average ms per launch from HIP events on the launch stream, after one untimed launch."""
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


HOST_REPS = 3   # host-inclusive runs timed per config (after one untimed full run); the median is reported


def _median_secs(fn, reps):
    """Median wall seconds of `reps` calls of fn (host-inclusive paths: one call is a whole 4 GiB job)."""
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def _spot(crcs, frame_bytes, idx):
    """Number of sampled frames whose GPU CRC differs from zlib.crc32 (= ether_fcs)."""
    import zlib
    return sum(int(zlib.crc32(frame_bytes(int(i))) != int(crcs[int(i)])) for i in idx)


def extra_configs(torch, na, dev, stream, reps=5, host_gib=4.0):
    """BASELINE configs[2] (IMIX), configs[3] (jumbo) and the host-inclusive rate, one after the other
    in HBM (each freed before the next), timed like the headline. Returns a dict for the JSON line."""
    import numpy as np
    rng = np.random.default_rng(2026)
    res = {}
    # ---- configs[2]: 128 M IMIX frames, 7:4:1 of 64/576/1518 in exact counts, shuffled, packed ----
    n = 128 << 20
    ln_np = imix_lengths(n)   # 78293676 / 44739242 / 11184810 frames of 64 / 576 / 1518 B
    ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
    off = torch.zeros(n, dtype=torch.int64, device=dev)
    off[1:] = torch.cumsum(ln[:-1].to(torch.int64), 0)
    total = int(off[-1].item()) + int(ln_np[-1])
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, total, SEED + 2, 0, stream)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ms = _time_launches(lambda: na.batch_dev(arena, total, off, ln, out, n, stream), reps, stream, torch)
    crcs = out.cpu().numpy().view(np.uint32)
    # the arena-stream kernel's own load ceiling: the same units, items, slot DMA and schedule
    # without marks, chain, contributions or closes (fcs_stream_load_dev)
    lsink = torch.zeros(4, dtype=torch.int32, device=dev)
    load_ms = _time_launches(lambda: na.stream_load_dev(arena, total, off, ln, n, lsink, stream), reps, stream, torch)
    offs = off.cpu().numpy()
    idx = rng.integers(0, n, 256)
    bad = _spot(crcs, lambda i: splitmix_bytes(SEED + 2, int(offs[i]), int(ln_np[i])).tobytes(), idx)
    gbs = total / ms / 1e6
    pmc = _load_pmc_traffic(n, "imix")
    res["imix_128M"] = {"config": "BASELINE configs[2]", "frames": n, "bytes": total, "ms": round(ms, 4),
                        "GB_s": round(gbs, 1), "GiB_s": round(total / ms / 1e-3 / GIB, 1),
                        "Gframes_s": round(n / ms / 1e6, 3), "metadata_bytes": n * 12,
                        "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                     "frac": round(gbs / HBM_PEAK_GBS, 4), "traffic": pmc[0] if pmc else None,
                                     "traffic_source": pmc[1] if pmc else None,
                                     "stream_load_ms": round(load_ms, 4),
                                     "stream_load_gbs": round(total / load_ms / 1e6, 1),
                                     "frac_of_stream_load": round(load_ms / ms, 4)},
                        "spot_checked": len(idx), "spot_bad": bad}
    del arena, out, off, ln, crcs, offs, ln_np, lsink
    torch.cuda.empty_cache()
    # ---- configs[3]: 16 M x 9000-B jumbo frames ----
    n, L = 16 << 20, 9000
    arena = torch.empty(n * L, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, n * L, SEED + 3, 0, stream)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ms = _time_launches(lambda: na.fixed_dev(arena, L, L, n, out, stream), reps, stream, torch)
    crcs = out.cpu().numpy().view(np.uint32)
    idx = rng.integers(0, n, 128)
    bad = _spot(crcs, lambda i: splitmix_bytes(SEED + 3, i * L, L).tobytes(), idx)
    gbs = n * L / ms / 1e6
    pmc = _load_pmc_traffic(n, L)
    res["jumbo_16M_x_9000"] = {"config": "BASELINE configs[3]", "frames": n, "bytes": n * L, "ms": round(ms, 4),
                               "GB_s": round(gbs, 1), "GiB_s": round(n * L / ms / 1e-3 / GIB, 1),
                               "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                                            "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4),
                                            "traffic": pmc[0] if pmc else None,
                                            "traffic_source": pmc[1] if pmc else None},
                               "spot_checked": len(idx), "spot_bad": bad}
    del arena, out, crcs
    torch.cuda.empty_cache()
    # ---- host-inclusive: 1518-B frames in pinned host memory, through ether_fcs_fixed_host ----
    L = 1518
    n = int(host_gib * GIB) // L
    nbytes = n * L
    lib = na.load()
    p = lib.fcs_host_alloc(nbytes)
    if p:
        pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(d, nbytes, SEED + 4, 0, stream)
        torch.cuda.synchronize()
        torch.from_numpy(pinned).copy_(d)   # D2H straight into the pinned arena (no pageable staging copy)
        del d
        torch.cuda.empty_cache()
        hout = np.zeros(n, dtype=np.uint32)
        na.fixed_host(p, L, L, n, hout)     # untimed: every pipeline buffer and stream allocated
        secs = _median_secs(lambda: na.fixed_host(p, L, L, n, hout), HOST_REPS)
        idx = rng.integers(0, n, 128)
        bad = _spot(hout, lambda i: pinned[i * L:(i + 1) * L].tobytes(), idx)
        # the measured ceiling: plain async H2D copies of the same pinned arena, 1 GiB at a time
        src = torch.from_numpy(pinned)
        chunk = min(nbytes, int(GIB))
        dbuf = torch.empty(chunk, dtype=torch.uint8, device=dev)
        dbuf.copy_(src[:chunk], non_blocking=True)
        torch.cuda.synchronize()

        def copies():
            for o in range(0, nbytes, chunk):
                m = min(chunk, nbytes - o)
                dbuf[:m].copy_(src[o:o + m], non_blocking=True)
            torch.cuda.synchronize()
        h2d = nbytes / _median_secs(copies, HOST_REPS) / 1e9
        del dbuf, src
        torch.cuda.empty_cache()
        res["host_inclusive_1518"] = {"what": "pinned host frames -> chunked H2D -> kernel -> D2H of CRCs "
                                              "(ether_fcs_fixed_host); PCIe Gen5 x16 bound, never `value`",
                                      "frames": n, "bytes": nbytes, "ms": round(secs * 1e3, 3),
                                      "timed_runs": HOST_REPS, "stat": "median after one untimed full run",
                                      "GB_s": round(nbytes / secs / 1e9, 2), "GiB_s": round(nbytes / secs / GIB, 2),
                                      "roofline": {"bound": "pcie", "achieved": round(nbytes / secs / 1e9, 2),
                                                   "peak": 63.0, "unit": "GB/s",
                                                   "frac": round(nbytes / secs / 1e9 / 63.0, 4),
                                                   "h2d_copy_gbs": round(h2d, 2),
                                                   "frac_of_h2d_copy": round(nbytes / secs / 1e9 / h2d, 4)},
                                      "spot_checked": len(idx), "spot_bad": bad}
        del pinned, hout
        lib.fcs_host_free(p)
    # ---- host-inclusive IMIX: the same 7:4:1 mix in pinned host memory, offsets and lengths in
    #      pageable host arrays, through ether_fcs_batch_host (north_star: "the rate including the
    #      copies to and from the GPU") ----
    res["host_inclusive_imix"] = host_inclusive_imix(torch, na, dev, stream, rng, host_gib)
    return res


def imix_lengths(n: int, seed: int = 7):
    """BASELINE configs[2]: n frames of 64/576/1518 B in exact 7:4:1 proportions, shuffled."""
    import numpy as np
    c1518 = n // 12
    c576 = (n * 4) // 12
    c64 = n - c576 - c1518
    ln = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), [c64, c576, c1518])
    np.random.default_rng(seed).shuffle(ln)
    return ln


def host_inclusive_imix(torch, na, dev, stream, rng, host_gib=4.0):
    """IMIX frames packed in a pinned host arena (fcs_host_alloc) -> ether_fcs_batch_host (chunked H2D
    of frames + offsets + lengths -> arena-stream kernel -> D2H of the CRCs). Ceiling: plain async H2D copies
    of the same pinned arena plus the 12 B of metadata per frame, same process."""
    import numpy as np
    n = int(host_gib * GIB / 355.83)   # frames whose mean length is 4270 / 12 B
    ln = imix_lengths(n, seed=11)
    off = np.zeros(n, dtype=np.uint64)
    np.cumsum(ln[:-1], dtype=np.uint64, out=off[1:])
    total = int(off[-1]) + int(ln[-1])
    lib = na.load()
    p = lib.fcs_host_alloc(total)
    if not p:
        return None
    try:
        pinned = np.ctypeslib.as_array((ctypes.c_uint8 * total).from_address(p))
        d = torch.empty(total, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(d, total, SEED + 5, 0, stream)
        torch.cuda.synchronize()
        torch.from_numpy(pinned).copy_(d)   # D2H straight into the pinned arena (no pageable staging copy)
        del d
        torch.cuda.empty_cache()
        out = np.zeros(n, dtype=np.uint32)
        na.batch_host(p, total, off, ln, out, n)   # untimed: every pipeline buffer and stream allocated
        secs = _median_secs(lambda: na.batch_host(p, total, off, ln, out, n), HOST_REPS)
        idx = rng.integers(0, n, 128)
        bad = _spot(out, lambda i: pinned[int(off[i]):int(off[i]) + int(ln[i])].tobytes(), idx)
        src = torch.from_numpy(pinned)
        meta = torch.from_numpy(np.concatenate([off.view(np.uint8), ln.view(np.uint8)])).pin_memory()
        chunk = min(total, int(GIB))
        dbuf = torch.empty(chunk, dtype=torch.uint8, device=dev)
        dmeta = torch.empty(meta.numel(), dtype=torch.uint8, device=dev)
        dbuf.copy_(src[:chunk], non_blocking=True)
        torch.cuda.synchronize()

        def copies():
            for o in range(0, total, chunk):
                k = min(chunk, total - o)
                dbuf[:k].copy_(src[o:o + k], non_blocking=True)
            dmeta.copy_(meta, non_blocking=True)
            torch.cuda.synchronize()
        copy_secs = _median_secs(copies, HOST_REPS)
        del dbuf, dmeta, src, meta
        torch.cuda.empty_cache()
        gbs = total / secs / 1e9
        return {"what": "IMIX frames in pinned host memory + offsets/lengths in pageable host arrays -> "
                        "ether_fcs_batch_host (chunked H2D -> arena-stream kernel -> D2H of CRCs); PCIe bound, never `value`",
                "frames": n, "bytes": total, "metadata_bytes": n * 12, "ms": round(secs * 1e3, 3),
                "timed_runs": HOST_REPS, "stat": "median after one untimed full run",
                "GB_s": round(gbs, 2), "Mframes_s": round(n / secs / 1e6, 1),
                "roofline": {"bound": "pcie", "achieved": round(gbs, 2), "peak": 63.0, "unit": "GB/s",
                             "frac": round(gbs / 63.0, 4),
                             "h2d_copy_s": round(copy_secs, 4),
                             "frac_of_h2d_copy": round(copy_secs / secs, 4),
                             "h2d_copy_what": "plain async copies of the pinned arena (1 GiB pieces) plus the "
                                              "pinned offsets and lengths, same process"},
                "spot_checked": len(idx), "spot_bad": bad}
    finally:
        lib.fcs_host_free(p)


def imix_shard(world: int, rank: int, n_blk: int):
    """Host side of imix_sharded: rank's contiguous frame range [lo, hi) of the global IMIX stream
    (`world` blocks of n_blk frames) from fcs_shard_plan over the global lengths, the shard's lengths
    and offsets (packed, from 0), the global byte position of its first byte, and its byte count."""
    import numpy as np
    blk = imix_lengths(n_blk)
    blk_bytes = int(blk.sum(dtype=np.uint64))
    glob_len = np.tile(blk, world)
    lo, hi = shard_range(len(glob_len), world, rank, glob_len)
    del glob_len
    idx = np.arange(lo, hi, dtype=np.int64) % n_blk
    ln_np = blk[idx]
    del idx
    q, r = divmod(lo, n_blk)
    byte0 = q * blk_bytes + int(blk[:r].sum(dtype=np.uint64))
    off_np = np.zeros(hi - lo, dtype=np.uint64)
    if hi - lo > 1:
        np.cumsum(ln_np[:-1], dtype=np.uint64, out=off_np[1:])
    total = int(off_np[-1]) + int(ln_np[-1]) if hi > lo else 0
    return lo, hi, ln_np, off_np, byte0, total


def imix_sharded(torch, na, dev, stream, world: int, rank: int, dist, n_blk: int = 128 << 20, reps: int = 5):
    """BASELINE configs[2] per GPU at N > 1 (weak scaling): the global stream is `world` blocks of n_blk
    IMIX frames (64/576/1518 B, 7:4:1, shuffled), packed. Each rank takes its byte-balanced contiguous
    shard from the engine's planner (fcs_shard_plan over the global lengths), fills it with its slice
    of one global byte stream, and times `reps` launches of ether_fcs_batch_dev with HIP events on its
    stream; rank 0 reports the aggregate (all ranks' bytes / the slowest rank's time). Only the
    barrier, the max and two integer sums cross ranks (gloo)."""
    import numpy as np
    lo, hi, ln_np, off_np, byte0, total = imix_shard(world, rank, n_blk)
    n = hi - lo
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, total, SEED + 2, byte0, stream)
    off = torch.from_numpy(off_np.view(np.int64)).to(dev)
    ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    na.batch_dev(arena, total, off, ln, out, n, stream)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        na.batch_dev(arena, total, off, ln, out, n, stream)
    e1.record(stream)
    torch.cuda.synchronize()
    dist.barrier()
    wall = time.perf_counter() - t0
    kms = e0.elapsed_time(e1) / reps
    rng = np.random.default_rng(100 + rank)
    pick = rng.integers(0, n, 64)
    crcs = out.cpu().numpy().view(np.uint32)
    bad = _spot(crcs, lambda i: splitmix_bytes(SEED + 2, byte0 + int(off_np[i]), int(ln_np[i])).tobytes(), pick)
    agg = torch.tensor([total, n, bad], dtype=torch.int64)
    dist.all_reduce(agg)
    tmax = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    del arena, off, ln, out
    torch.cuda.empty_cache()
    all_bytes, all_frames, all_bad = (int(x) for x in agg.tolist())
    t = float(tmax.item()) / reps
    return {"config": "BASELINE configs[2] per GPU, weak scaling", "frames_per_block": n_blk, "blocks": world,
            "global_frames": all_frames, "global_bytes": all_bytes, "ms_per_step_max_rank": round(t * 1e3, 4),
            "GB_s_aggregate": round(all_bytes / t / 1e9, 1), "rank0_kernel_ms": round(kms, 4),
            "rank0_frames": n, "rank0_bytes": total,
            "sharding": "fcs_shard_plan byte-balanced over the global lengths (contiguous ranges)",
            "spot_checked": 64 * world, "spot_bad": all_bad}


def host_aggregate(per_rank, rep_max_secs):
    """Whole-job host-inclusive rate at N > 1: per_rank = [{"rank", "bytes", "secs"}] (each rank's median
    of its own timed runs), rep_max_secs = per timed run, the slowest rank's time. The aggregate is all
    ranks' bytes over the median of those per-run maxima (the ranks run concurrently, barrier between
    runs), as `value` is all ranks' bytes over the slowest rank."""
    total = sum(int(r["bytes"]) for r in per_rank)
    t = sorted(rep_max_secs)[len(rep_max_secs) // 2]
    return {"GB_s_aggregate": round(total / t / 1e9, 2), "bytes_all_ranks": total,
            "secs_max_rank": round(t, 4),
            "per_rank": [{"rank": int(r["rank"]), "bytes": int(r["bytes"]), "secs": round(float(r["secs"]), 4),
                          "GB_s": round(int(r["bytes"]) / float(r["secs"]) / 1e9, 2)}
                         for r in sorted(per_rank, key=lambda r: r["rank"])]}


def gather_host_times(torch, dist, world: int, rank: int, nbytes: int, secs, bad: int):
    """Cross-rank part of host_inclusive_sharded (gloo, host values only): every rank's (bytes, median
    of its runs, spot-check misses), and per timed run the slowest rank's time."""
    rep_max = torch.tensor(list(secs), dtype=torch.float64)
    dist.all_reduce(rep_max, op=dist.ReduceOp.MAX)
    mine = {"rank": rank, "bytes": int(nbytes), "secs": sorted(secs)[len(secs) // 2], "spot_bad": int(bad)}
    allr = [None] * world
    dist.all_gather_object(allr, mine)
    return allr, rep_max.tolist()


def host_inclusive_sharded(torch, na, dev, stream, world: int, rank: int, dist, host_gib: float = 4.0):
    """The host-inclusive rate at N > 1 (bounded by each GPU's PCIe link
    and the host's DRAM): every rank checksums its own host_gib of 1518-B frames in pinned host memory
    through ether_fcs_fixed_host (chunked H2D -> kernel -> D2H), all ranks at once, HOST_REPS timed
    runs after one untimed one with a barrier before each. Rank 0 reports each rank's rate and the
    aggregate over the slowest rank (host_aggregate)."""
    import numpy as np
    L = 1518
    n = int(host_gib * GIB) // L
    nbytes = n * L
    lib = na.load()
    p = lib.fcs_host_alloc(nbytes)
    ok = torch.tensor([1 if p else 0], dtype=torch.int64)
    dist.all_reduce(ok, op=dist.ReduceOp.MIN)
    if not int(ok.item()):
        if p:
            lib.fcs_host_free(p)
        return None
    try:
        pinned = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(p))
        d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
        na.fill_splitmix_dev(d, nbytes, SEED + 6, rank * nbytes, stream)   # this rank's slice of one stream
        torch.cuda.synchronize()
        torch.from_numpy(pinned).copy_(d)   # D2H straight into the pinned arena (no pageable staging copy)
        del d
        torch.cuda.empty_cache()
        hout = np.zeros(n, dtype=np.uint32)
        na.fixed_host(p, L, L, n, hout)   # untimed: pipeline buffers and streams allocated
        secs = []
        for _ in range(HOST_REPS):
            dist.barrier()
            t0 = time.perf_counter()
            na.fixed_host(p, L, L, n, hout)
            secs.append(time.perf_counter() - t0)
        idx = np.random.default_rng(200 + rank).integers(0, n, 64)
        bad = _spot(hout, lambda i: pinned[i * L:(i + 1) * L].tobytes(), idx)
        allr, rep_max = gather_host_times(torch, dist, world, rank, nbytes, secs, bad)
        del pinned, hout
    finally:
        lib.fcs_host_free(p)
    agg = host_aggregate(allr, rep_max)
    agg.update({"what": "each rank: its own pinned host slice of 1518-B frames -> ether_fcs_fixed_host "
                        "(chunked H2D -> kernel -> D2H of CRCs), all ranks at once; PCIe bound, never `value`",
                "frames_per_rank": n, "timed_runs": HOST_REPS,
                "stat": "median over runs of the slowest rank's time (barrier before each run)",
                "spot_checked": 64 * world, "spot_bad": sum(int(r["spot_bad"]) for r in allr)})
    return agg


def cpu_baseline(frames: int = 1 << 20, L: int = 1518):
    """Oracle restatement of ether_fcs (src/ether_fcs.c:4-19) on the SURVEY §8d dataset."""
    import numpy as np
    here = os.path.join(ROOT, "oracle", "_build")
    res = {}
    buf = np.empty(frames * L, dtype=np.uint8)
    out = np.empty(frames, dtype=np.uint32)
    for tag, so in (("O2", "liboracle.so"), ("O0", "liboracle_O0.so")):
        path = os.path.join(here, so)
        if not os.path.exists(path):
            continue
        o = ctypes.CDLL(path)
        o.oracle_xorshift64_fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint64)]
        o.oracle_time_fixed.restype = ctypes.c_double
        o.oracle_time_fixed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_size_t,
                                        ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
        if "gen" not in res:
            st = ctypes.c_uint64(42)
            o.oracle_xorshift64_fill(buf.ctypes.data, buf.size, ctypes.byref(st))
            res["gen"] = True
        secs = o.oracle_time_fixed(buf.ctypes.data, L, L, frames, out.ctypes.data, 0, 1)
        x = int(np.bitwise_xor.reduce(out))
        res[tag] = {"gibs": frames * L / secs / GIB, "secs": secs, "xor": x}
        if tag == "O2":   # secondary figure: the same loop on the 16 host cores a GPU box grants
            secs16 = o.oracle_time_fixed(buf.ctypes.data, L, L, frames, out.ctypes.data, 0, 16)
            res["all"] = {"gibs": frames * L / secs16 / GIB, "threads": 16}
    # the reference's own src/ether_fcs.c (oracle/_ref, built from /root/reference at the reference
    # Makefile's flags -O0 -g -std=gnu99), called once per frame by the oracle's timing loop
    ref_path = os.path.join(ROOT, "oracle", "_ref", "libref_fcs.so")
    if "O2" in res and os.path.exists(ref_path):
        r = ctypes.CDLL(ref_path)
        o = ctypes.CDLL(os.path.join(here, "liboracle.so"))
        FN = ctypes.CFUNCTYPE(ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t)
        o.oracle_time_calls.restype = ctypes.c_double
        o.oracle_time_calls.argtypes = [FN, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_size_t,
                                        ctypes.c_void_p]
        fn = ctypes.cast(r.ether_fcs, FN)
        secs = o.oracle_time_calls(fn, buf.ctypes.data, L, L, frames, out.ctypes.data)
        res["ref"] = {"gibs": frames * L / secs / GIB, "secs": secs, "xor": int(np.bitwise_xor.reduce(out))}
    if "O2" not in res:
        return None
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    ok = res["O2"]["xor"] == 0x600A585E
    sample = (f"{frames} x {L}-B frames (xorshift64 seed 42, SURVEY §8d), oracle nibble-table "
              f"restatement of src/ether_fcs.c, 1 host thread; -O2 {res['O2']['secs']:.2f} s"
              + (f"; reference flags -O0 -g: {res['O0']['gibs']:.4f} GiB/s ({res['O0']['secs']:.2f} s)"
                 if "O0" in res else "")
              + f"; XOR of CRCs 0x{res['O2']['xor']:08X} ({'ok' if ok else 'MISMATCH'}); host CPU: {cpu_model}; "
              f"nproc {os.cpu_count()}")
    if "ref" in res:   # the reference itself is the baseline; the port's figures stay beside it
        ref_ok = res["ref"]["xor"] == 0x600A585E
        sample = (f"{frames} x {L}-B frames (xorshift64 seed 42, SURVEY §8d), the reference's own "
                  f"src/ether_fcs.c compiled at its Makefile flags (-O0 -g -std=gnu99; oracle/_ref), one "
                  f"ether_fcs call per frame on 1 host thread: {res['ref']['secs']:.2f} s; XOR of CRCs "
                  f"0x{res['ref']['xor']:08X} ({'ok' if ref_ok else 'MISMATCH'}). Beside it, the oracle port: "
                  + sample)
        return {"value": round(res["ref"]["gibs"], 4), "unit": "GiB/s", "cores": 1, "kind": "reference",
                "sample": sample, "value_port_O2": round(res["O2"]["gibs"], 4),
                "value_port_O0": round(res["O0"]["gibs"], 4) if "O0" in res else None,
                "value_port_16_threads": round(res["all"]["gibs"], 4)}
    return {"value": round(res["O2"]["gibs"], 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": sample, "value_O0": round(res["O0"]["gibs"], 4) if "O0" in res else None,
            "value_16_threads": round(res["all"]["gibs"], 4)}


def _free_port() -> int:
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(gpus: int, argv) -> int:
    """`bench.py --gpus N` started without a launcher: start N rank processes of this script under
    torch.distributed.run (one per GPU, rendezvous on 127.0.0.1) from this parent, which has made no
    GPU call, and return their exit status. The ranks print the one JSON line (rank 0)."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def device_entry(rank: int, local: int, torch, dry_run: bool):
    """This rank's device identity for config.devices: HIP ordinal and PCI address (domain:bus:device)."""
    if dry_run:
        return {"rank": rank, "local_rank": local, "hip_device": None, "pci": None, "name": "dry-run (no GPU)"}
    d = torch.cuda.current_device()
    p = torch.cuda.get_device_properties(d)
    pci = f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}"
    return {"rank": rank, "local_rank": local, "hip_device": d, "pci": pci, "name": p.name,
            "uuid": str(getattr(p, "uuid", ""))}


def label_devices(entries):
    """Mark ranks that share a physical GPU (a rehearsal of the N > 1 path on a smaller box)."""
    seen = {}
    for e in entries:
        key = e.get("pci") or f"dry{e['rank']}"
        seen.setdefault(key, []).append(e["rank"])
    for e in entries:
        key = e.get("pci") or f"dry{e['rank']}"
        e["shares_gpu_with_ranks"] = [r for r in seen[key] if r != e["rank"]]
    return entries, len(seen)


def dry_run(args, world: int, rank: int, local: int) -> None:
    """--dry-run: the launch and rendezvous only (gloo, no GPU call), for the CPU tests of --gpus."""
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    entries = [device_entry(rank, local, torch, True)]
    if dist:
        allv = [None] * world
        dist.all_gather_object(allv, entries[0])
        entries = allv
        dist.barrier()
    if rank == 0:
        devs, distinct = label_devices(entries)
        print(json.dumps({"metric": METRIC, "value": None, "unit": "GiB/s", "n_gpus": world, "dry_run": True,
                          "config": {"devices": devs, "distinct_devices": distinct}}), flush=True)
    if dist:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs (ranks). Without WORLD_SIZE in the environment and N > 1, bench.py starts the N "
                         "ranks itself (torch.distributed.run); with WORLD_SIZE set it must equal N")
    ap.add_argument("--dry-run", action="store_true", help="launch and rendezvous only, no GPU (CPU tests)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--frames-per-gpu", type=int, default=64 << 20)
    ap.add_argument("--len", type=int, default=1518)
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--no-configs", action="store_true", help="skip the other BASELINE configs")
    ap.add_argument("--imix-frames-per-gpu", type=int, default=128 << 20,
                    help="N > 1: IMIX frames per GPU of the sharded configs[2] run (0 = skip)")
    ap.add_argument("--host-gib-per-gpu", type=float, default=4.0,
                    help="N > 1: GiB of pinned host frames per rank for the host-inclusive run (0 = skip)")
    args = ap.parse_args()

    # --gpus is authoritative: no launcher -> start the ranks here, before any
    # GPU call in this process; a launcher whose world size disagrees -> refuse
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to time a different "
              "number of GPUs than asked", file=sys.stderr, flush=True)
        sys.exit(1)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run(args, world, rank, local)
        return

    import numpy as np
    import torch
    import nstack_amd as na

    dist = None
    if world > 1:
        # gloo on the host: the barrier and the 8-byte max-over-ranks of the elapsed time are the
        # only cross-rank traffic; frames never leave their GPU (no RCCL, BASELINE north_star)
        import torch.distributed as dist
        # one GPU per rank; on a box with fewer GPUs than ranks (a rehearsal of the N > 1 path)
        # ranks share them round-robin
        torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    na.load()
    devices = [device_entry(rank, local, torch, False)]
    if dist:   # every rank's HIP device and PCI address, so a SCALE line shows N distinct GPUs
        allv = [None] * world
        dist.all_gather_object(allv, devices[0])
        devices = allv
    devices, distinct = label_devices(devices)

    L = args.len
    F = args.frames_per_gpu
    total = F * world
    lo, hi = shard_range(total, world, rank)
    n = hi - lo
    nbytes = n * L
    stream = torch.cuda.current_stream()

    # Synthetic frames: this rank's slice of one global counter-based byte stream.
    arena = torch.empty(nbytes + 64, dtype=torch.uint8, device=dev)
    na.fill_splitmix_dev(arena, nbytes, SEED, lo * L, stream)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()

    def step():
        na.fixed_dev(arena, L, L, n, out, stream)

    # ---- read-stream ceiling over the same buffer: untimed calibration, also warms the memory
    #      system and clocks before the warmup steps ----
    rs = torch.cuda.Event(enable_timing=True)
    re_ = torch.cuda.Event(enable_timing=True)
    na.read_stream_dev(arena, nbytes, sink, stream)
    rs.record(stream)
    for _ in range(5):
        na.read_stream_dev(arena, nbytes, sink, stream)
    re_.record(stream)
    torch.cuda.synchronize()
    read_ms = rs.elapsed_time(re_) / 5
    read_gbs = nbytes / (read_ms * 1e-3) / 1e9
    # the LDS-DMA read ceiling: the headline kernel's own loads and schedule without the CRC work
    na.dma_stream_dev(arena, nbytes, sink, stream)
    rs.record(stream)
    for _ in range(5):
        na.dma_stream_dev(arena, nbytes, sink, stream)
    re_.record(stream)
    torch.cuda.synchronize()
    dma_gbs = nbytes / (rs.elapsed_time(re_) / 5 * 1e-3) / 1e9


    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()

    # ---- timed region: exactly K steps, barrier + synchronize on both sides ----
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    wall = t1 - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps   # HIP events on the launch stream

    times = torch.tensor([wall], dtype=torch.float64)
    if dist:
        dist.all_reduce(times, op=dist.ReduceOp.MAX)
    tmax = float(times.item())
    total_bytes = total * L
    value = total_bytes * args.steps / tmax / GIB

    # ---- spot check of this rank's output: sampled frames re-created on the host, checked with
    #      zlib.crc32 (the stdlib CRC-32 = ether_fcs; the oracle is only for the CPU-baseline leg) ----
    verified = None
    if not args.no_verify:
        import zlib
        crcs = out.cpu().numpy().view(np.uint32)
        rng = np.random.default_rng(rank)
        idx = np.unique(np.concatenate([rng.integers(0, n, 256), [0, n - 1]]))
        bad = 0
        for i in idx:
            frame = splitmix_bytes(SEED, (lo + int(i)) * L, L)
            bad += int(zlib.crc32(frame.tobytes()) != int(crcs[i]))
        flag = torch.tensor([bad], dtype=torch.int64)
        if dist:
            dist.all_reduce(flag)
        verified = int(flag.item()) == 0

    achieved_gbs = nbytes / (kernel_ms * 1e-3) / 1e9
    pmc = _load_pmc_traffic(n, L, "fcs_dma_kernel")
    roofline = {"bound": "hbm", "achieved": round(achieved_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved_gbs / HBM_PEAK_GBS, 4),
                "traffic": pmc[0] if pmc else None,
                "traffic_source": pmc[1] if pmc else None,
                "algorithmic_bytes_per_launch": nbytes,
                "kernel_ms_per_launch": round(kernel_ms, 4),
                "read_stream_gbs": round(read_gbs, 1),
                "frac_of_read_stream": round(achieved_gbs / read_gbs, 4),
                "dma_stream_gbs": round(dma_gbs, 1),
                "frac_of_dma_stream": round(achieved_gbs / dma_gbs, 4)}
    prof = _load_kernel_profile("void fcs::fcs_dma_kernel<2, false>", nbytes) if L == 1518 and F == 64 << 20 else None
    if prof:   # the committed trace of this command (another box, under the tracer): box spread in DESIGN §4.2
        roofline.update(prof)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline()
    configs = None
    if world == 1 and not args.no_configs and F == 64 << 20 and L == 1518:
        del arena, out
        torch.cuda.empty_cache()
        configs = extra_configs(torch, na, dev, stream)
        for c in configs.values():   # the headline run's measured read ceilings, for comparison
            rf = c.get("roofline", {})
            if rf.get("bound") == "hbm":
                rf["frac_of_read_stream"] = round(rf["achieved"] / read_gbs, 4)
                rf["frac_of_dma_stream"] = round(rf["achieved"] / dma_gbs, 4)

    if dist and not args.no_configs and args.imix_frames_per_gpu > 0:
        del arena, out
        torch.cuda.empty_cache()
        configs = {"imix_sharded": imix_sharded(torch, na, dev, stream, world, rank, dist,
                                                n_blk=args.imix_frames_per_gpu)}
    if dist and not args.no_configs and args.host_gib_per_gpu > 0:
        if configs is None:
            del arena, out
            torch.cuda.empty_cache()
            configs = {}
        configs["host_inclusive_1518_sharded"] = host_inclusive_sharded(torch, na, dev, stream, world, rank, dist,
                                                                        host_gib=args.host_gib_per_gpu)
    if dist:
        dist.barrier()
    if rank == 0:
        rec = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(tmax / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: counter-based splitmix64 bytes (seed 0x{SEED:X}), frames packed at stride {L}",
            "config": {"workload": f"{F // (1 << 20)} M x {L}-B frames per GPU, one CRC-32 per frame, "
                                   "single HIP launch per step (BASELINE configs[1]; configs[4] at 8 GPUs)",
                       "frames_per_gpu": F, "frame_len": L, "global_frames": total,
                       "parallelism": f"frames sharded over {world} GPU(s), no collective on the data path",
                       "devices": devices, "distinct_devices": distinct},
            "pct_hbm_peak": round(100.0 * value * GIB / 1e9 / world / HBM_PEAK_GBS, 2),
            "verified": verified,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "configs": configs,
            "engine": na.version(),
        }
        print(json.dumps(rec), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
