#!/usr/bin/env python3
"""FCS of every frame of a pcap capture on the GPU, or RX verification of a
capture taken with FCS trailers (e.g. `ethtool -K <if> rx-fcs on`).

    python tools/pcap_fcs.py capture.pcap [--verify] [--crc-out crcs.txt] [--add-fcs out.pcap]

Prints one JSON line: frames, bytes, link type, truncated records, and either a digest of the
FCS values (XOR and 64-bit sum) or the number of frames failing the residue check with their
indices (first 20). Truncated records (snap length) are reported; their FCS cannot be checked.
--add-fcs writes a copy of the capture with every frame followed by its FCS, computed on the GPU
exactly as ether_send places it (src/linux/ether.c:262-263): captures taken on veth or AF_PACKET
carry no trailer; the copy is what the wire would carry and passes --verify.
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
    ap.add_argument("--add-fcs", metavar="OUT", help="write the capture with FCS trailers appended")
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
    if a.add_fcs and n:
        rec["with_fcs"] = a.add_fcs
        add_fcs(arena, off, ln, a.add_fcs, lt)
    rec["seconds"] = round(time.perf_counter() - t0, 4)
    print(json.dumps(rec))


def add_fcs(arena, off, ln, out_path, linktype=1):
    """Write frames (arena, off, len) as a pcap with each frame's FCS appended: the frames are
    respaced with 4 spare bytes after each, ether_fcs_tx_batch_host fills them on the GPU."""
    import numpy as np
    import nstack_amd as na
    n = len(ln)
    ln = np.asarray(ln, dtype=np.uint32)
    off2 = np.zeros(n, dtype=np.uint64)
    off2[1:] = np.cumsum(ln[:-1].astype(np.uint64) + 4)
    total = int(off2[-1]) + int(ln[-1]) + 4 if n else 0
    out = np.zeros(max(total, 1), dtype=np.uint8)
    for i in range(n):   # respacing only; the FCS itself comes from the GPU
        o, L = int(off[i]), int(ln[i])
        out[int(off2[i]):int(off2[i]) + L] = arena[o:o + L]
    if n:
        na.tx_batch_host(out, total, off2, ln, n)
    na.pcap_write(out_path, out, off2, ln + 4, linktype)


if __name__ == "__main__":
    main()
