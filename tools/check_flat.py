#!/usr/bin/env python3
"""Parity spot check of a library variant against zlib (measurement tool): fixed short frames and an
IMIX batch through the flat (windowed) paths, every frame compared; with --lens L1,L2,... fixed-length
batches of those lengths instead (gaps 0 and 8, odd base), e.g. jumbo frames for the segment kernels.
usage: NSTACK_FCS_LIB=... check_flat.py [--lens 9000,16500]"""
import numpy as np
import torch
import zlib
import sys
sys.path.insert(0, ".")
import nstack_amd as na

torch.cuda.set_device(0)
na.load()
dev = torch.device("cuda:0")
bad_total = 0
if len(sys.argv) > 2 and sys.argv[1] == "--lens":
    for L in (int(x) for x in sys.argv[2].split(",")):
        for gap in (0, 8):
            stride = L + gap
            n = max(64, (96 << 20) // stride)
            host = np.random.default_rng(L + gap).integers(0, 256, n * stride + 64, dtype=np.uint8)
            d = torch.from_numpy(host).to(dev)
            out = torch.empty(n, dtype=torch.int32, device=dev)
            na.fixed_dev(d.data_ptr() + 3, stride, L, n, out)
            torch.cuda.synchronize()
            got = out.cpu().numpy().view(np.uint32)
            exp = np.array([zlib.crc32(host[3 + i * stride:3 + i * stride + L].tobytes()) for i in range(n)],
                           dtype=np.uint32)
            bad = int((got != exp).sum())
            bad_total += bad
            print("fixed", L, "stride", stride, "n", n, "bad", bad, flush=True)
    sys.exit(1 if bad_total else 0)
for L in (64, 100, 576, 1000, 1503):
    n = 40000
    host = np.random.default_rng(L).integers(0, 256, n * L + 64, dtype=np.uint8)
    d = torch.from_numpy(host).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    na.fixed_dev(d.data_ptr() + 16, L, L, n, out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    exp = np.array([zlib.crc32(host[16 + i * L:16 + i * L + L].tobytes()) for i in range(n)], dtype=np.uint32)
    bad = int((got != exp).sum())
    bad_total += bad
    print("fixed", L, "bad", bad, flush=True)
rng = np.random.default_rng(3)
n = 100000
ln = rng.choice(np.array([64] * 7 + [576] * 4 + [1518] * 1 + [0, 1, 2000], dtype=np.uint32), n)
off = np.zeros(n, dtype=np.uint64)
off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
total = int(off[-1]) + int(ln[-1])
arena = rng.integers(0, 256, total + 8, dtype=np.uint8)
da = torch.from_numpy(arena).to(dev)
doff = torch.from_numpy(off.view(np.int64)).to(dev)
dln = torch.from_numpy(ln.view(np.int32)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
na.batch_dev(da, total, doff, dln, out, n)
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.uint32)
exp = np.array([zlib.crc32(arena[int(o):int(o) + int(l)].tobytes()) for o, l in zip(off, ln)], dtype=np.uint32)
bad = int((got != exp).sum())
bad_total += bad
print("imix+", "bad", bad, flush=True)
sys.exit(1 if bad_total else 0)
