#!/usr/bin/env python3
"""FCS of every frame of a pcap capture on the GPU, or RX verification of a
capture taken with FCS trailers (e.g. `ethtool -K <if> rx-fcs on`).

    python tools/pcap_fcs.py capture.pcap [--verify] [--crc-out crcs.txt]

Prints one JSON line: frames, bytes, link type, truncated records, and either a digest of the
FCS values (XOR and 64-bit sum) or the number of frames failing the residue check with their
indices (first 20). Truncated records (snap length) are reported; their FCS cannot be checked.
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pcap")
    ap.add_argument("--verify", action="store_true", help="frames carry their FCS: residue check")
    ap.add_argument("--crc-out", help="write one hex FCS per line")
    a = ap.parse_args()
    import numpy as np
    import nstack_amd as na
    n, nbytes, lt, trunc = na.pcap_scan(a.pcap)
    arena, off, ln, _ = na.pcap_read(a.pcap)
    rec = {"file": a.pcap, "frames": n, "bytes": nbytes, "linktype": lt, "truncated": trunc}
    t0 = time.perf_counter()
    if a.verify:
        ok = np.zeros(max(n, 1), dtype=np.uint8)
        bad = na.verify_host(arena, arena.nbytes, off, ln, ok, n) if n else 0
        rec.update(bad=bad, bad_frames=np.nonzero(ok[:n] == 0)[0][:20].tolist())
    else:
        out = np.zeros(max(n, 1), dtype=np.uint32)
        if n:
            na.batch_host(arena, arena.nbytes, off, ln, out, n)
        out = out[:n]
        rec.update(xor=f"0x{int(np.bitwise_xor.reduce(out)) if n else 0:08X}",
                   sum64=f"0x{int(out.astype(np.uint64).sum()) & (2**64 - 1):016X}")
        if a.crc_out:
            with open(a.crc_out, "w") as f:
                f.writelines(f"{int(c):08X}\n" for c in out)
    rec["seconds"] = round(time.perf_counter() - t0, 4)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
