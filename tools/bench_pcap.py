#!/usr/bin/env python3
"""Capture replay rate: a pcap of IMIX frames with FCS trailers, read into the
batch layout (include/nstack_pcap.h) and checked on the GPU.

    python tools/bench_pcap.py [--frames N] [--dir DIR]

Frames: 7:4:1 of 64/576/1518 B on the wire (covered 60/572/1514 B + 4-B FCS), random bytes,
shuffled; their trailers are written by ether_fcs_tx_batch_host. The file goes to DIR (default
$TMPDIR or /tmp) and is removed afterwards. Timed separately: fcs_pcap_scan, fcs_pcap_read
(page-cache-warm file: the first pass is untimed), ether_fcs_batch_host over the covered bytes,
and ether_fcs_verify_host over whole frames (residue check). Spot checks use zlib. Prints one
JSON line.
"""
import argparse
import json
import os
import sys
import tempfile
import time
import zlib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=4 << 20)
    ap.add_argument("--dir", default=os.environ.get("TMPDIR", "/tmp"))
    a = ap.parse_args()
    import numpy as np
    import nstack_amd as na

    m = a.frames
    counts = [m * 7 // 12, m * 4 // 12]
    counts.append(m - sum(counts))
    wire = np.repeat(np.array([64, 576, 1518], dtype=np.uint32), counts)
    np.random.default_rng(5).shuffle(wire)
    off = np.zeros(m, dtype=np.uint64)
    off[1:] = np.cumsum(wire[:-1], dtype=np.uint64)
    total = int(off[-1] + wire[-1])
    arena = np.random.default_rng(6).integers(0, 256, total, dtype=np.uint8)
    covered = (wire - 4).astype(np.uint32)
    na.tx_batch_host(arena, total, off, covered, m)

    fd, path = tempfile.mkstemp(suffix=".pcap", dir=a.dir)
    os.close(fd)
    res = {"frames": m, "bytes": total, "file_bytes": 24 + 16 * m + total}
    try:
        na.pcap_write(path, arena, off, wire)
        del arena
        na.pcap_read(path)                       # warm the page cache (untimed)
        t0 = time.perf_counter()
        n, nbytes, lt, trunc = na.pcap_scan(path)
        t1 = time.perf_counter()
        ar, o, ln, _ = na.pcap_read(path)
        t2 = time.perf_counter()
        assert n == m and nbytes == total and lt == 1 and trunc == 0
        out = np.zeros(n, dtype=np.uint32)
        cov = (ln - 4).astype(np.uint32)
        na.batch_host(ar, ar.nbytes, o, cov, out, n)      # warm the engine (untimed)
        t3 = time.perf_counter()
        na.batch_host(ar, ar.nbytes, o, cov, out, n)
        t4 = time.perf_counter()
        ok = np.zeros(n, dtype=np.uint8)
        bad = na.verify_host(ar, ar.nbytes, o, ln, ok, n)
        t5 = time.perf_counter()
        spot_bad = 0
        for i in np.random.default_rng(7).integers(0, n, 64):
            f = ar[int(o[i]):int(o[i]) + int(ln[i])].tobytes()
            spot_bad += int(zlib.crc32(f[:-4]) != int(out[i]) or f[-4:] != int(out[i]).to_bytes(4, "little"))
        res.update(
            scan_s=round(t1 - t0, 4), read_s=round(t2 - t1, 4), crc_s=round(t4 - t3, 4), verify_s=round(t5 - t4, 4),
            read_GB_s=round(res["file_bytes"] / (t2 - t1) / 1e9, 2),
            crc_GB_s=round(total / (t4 - t3) / 1e9, 2), crc_Mframes_s=round(n / (t4 - t3) / 1e6, 2),
            verify_GB_s=round(total / (t5 - t4) / 1e9, 2), verify_Mframes_s=round(n / (t5 - t4) / 1e6, 2),
            replay_GB_s=round(total / (t5 - t4 + t2 - t0) / 1e9, 2),
            bad=int(bad), spot_bad=spot_bad)
    finally:
        os.unlink(path)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
