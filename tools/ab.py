#!/usr/bin/env python3
"""In-process A/B timing of FCS kernel variants (measurement tool, not product code).

    python tools/ab.py [--frames F] [--len L] [--rounds R] lib1.so lib2.so ...

Every library is a full build of the engine (tools/variants.sh); all are loaded into ONE process
and launched round-robin on the same HBM-resident frames, so clock/device differences cancel
(cdna_hip_programming.md §5.4 rule 24). Prints median / min ms per launch and GB/s per variant,
and checks every variant's CRCs against the first one's.
"""
import argparse
import ctypes
import os
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--frames", type=int, default=64 << 20)
    ap.add_argument("--len", type=int, default=1518)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--what", default="fcs", help="comma list of fcs,stream,dma,stload,inet (stream: plain read "
                         "stream; dma: the LDS-DMA kernel's loads without the CRC work; stload (--imix): the "
                         "arena-stream kernel's loads and schedule without its CRC work; inet: ip_checksum, fixed)")
    ap.add_argument("--mix", default="64,576,1518:7,4,1",
                    help="with --imix: lengths:weights of the variable-length mix")
    ap.add_argument("--imix", action="store_true",
                    help="variable-length path: --frames IMIX frames (7:4:1 of 64/576/1518, shuffled)")
    a = ap.parse_args()
    import torch
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    n, L = a.frames, a.len
    libs = []
    for p in a.libs:
        lib = ctypes.CDLL(os.path.abspath(p))
        lib.ether_fcs_fixed_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                            ctypes.c_void_p, ctypes.c_void_p]
        lib.ether_fcs_batch_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        lib.fcs_read_stream_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        lib.fcs_dma_stream_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        lib.fcs_stream_load_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
        lib.inet_csum_fixed_dev.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        lib.inet_csum_batch_dev.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                            ctypes.c_void_p]
        lib.fcs_fill_splitmix64_dev.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                                                ctypes.c_void_p]
        libs.append(lib)
    if a.imix:
        import numpy as np
        rng = np.random.default_rng(7)
        lens_s, w_s = a.mix.split(":")
        pool = []
        for Lx, wx in zip(lens_s.split(","), w_s.split(",")):
            pool += [int(Lx)] * int(wx)
        ln_np = rng.choice(np.array(pool, dtype=np.uint32), n)
        ln = torch.from_numpy(ln_np.view(np.int32)).to(dev)
        off = torch.zeros(n, dtype=torch.int64, device=dev)
        off[1:] = torch.cumsum(ln[:-1].to(torch.int64), 0)
        total = int(off[-1].item()) + int(ln_np[-1])
    else:
        total = n * L
    arena = torch.empty(total, dtype=torch.uint8, device=dev)
    libs[0].fcs_fill_splitmix64_dev(arena.data_ptr(), total, 11, 0, None)
    outs = [torch.zeros(n, dtype=torch.int32, device=dev) for _ in libs]
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream()
    whats = a.what.replace("+", ",").split(",")   # "+" too: tools/gpu_run.sh turns commas into spaces
    times = {(w, i): [] for w in whats for i in range(len(libs))}

    def launch(w, i, lib):
        if w == "stream":
            return lib.fcs_read_stream_dev(arena.data_ptr(), total, sink.data_ptr(), st.cuda_stream)
        if w == "dma":
            return lib.fcs_dma_stream_dev(arena.data_ptr(), total, sink.data_ptr(), st.cuda_stream)
        if w == "stload":   # the arena-stream kernel's loads and schedule without its CRC work (--imix)
            return lib.fcs_stream_load_dev(arena.data_ptr(), total, off.data_ptr(), ln.data_ptr(), n,
                                           sink.data_ptr(), st.cuda_stream)
        if w == "inet" and a.imix:
            return lib.inet_csum_batch_dev(0, arena.data_ptr(), total, off.data_ptr(), ln.data_ptr(), None,
                                           outs[i].data_ptr(), n, st.cuda_stream)
        if w == "inet":
            return lib.inet_csum_fixed_dev(0, arena.data_ptr(), L, L, n, None, outs[i].data_ptr(), st.cuda_stream)
        if a.imix:
            return lib.ether_fcs_batch_dev(arena.data_ptr(), total, off.data_ptr(), ln.data_ptr(),
                                           outs[i].data_ptr(), n, st.cuda_stream)
        return lib.ether_fcs_fixed_dev(arena.data_ptr(), L, L, n, outs[i].data_ptr(), st.cuda_stream)

    res = {}
    for w in whats:
        for r in range(a.rounds + 1):
            for i, lib in enumerate(libs):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(a.reps):
                    rc = launch(w, i, lib)
                    assert rc == 0, rc
                e1.record(st)
                torch.cuda.synchronize()
                if r:
                    times[(w, i)].append(e0.elapsed_time(e1) / a.reps)
        for i, p in enumerate(a.libs):
            med, mn = statistics.median(times[(w, i)]), min(times[(w, i)])
            same = bool(torch.equal(outs[i], outs[0])) if w not in ("stream", "dma", "stload") else None
            print(f"{w:6s} {os.path.basename(p):28s} median {med:8.3f} ms  min {mn:8.3f} ms  "
                  f"{total / med / 1e6:8.1f} GB/s  same_as_first={same}", flush=True)

if __name__ == "__main__":
    main()
