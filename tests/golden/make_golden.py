"""Generate the golden fixtures in tests/golden/ from the REFERENCE itself.

Run in the build container only (needs /root/reference):

    make -C oracle ref && python tests/golden/make_golden.py

The expected values come from oracle/_ref/libref_fcs_O2.so, i.e. /root/reference/src/ether_fcs.c
(ether_fcs, src/ether_fcs.c:4-19) compiled unmodified by oracle/Makefile. zlib.crc32 is checked
alongside as an independent witness. Inputs are generated here from seeded generators, so the
fixtures are pure data: inputs (vectors.bin) + expected outputs (vectors.json, kat.json).
"""
import ctypes
import json
import os
import random
import struct
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_fcs_O2.so")
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle.so")


def load_ref():
    lib = ctypes.CDLL(REF_SO)
    lib.ether_fcs.restype = ctypes.c_uint32
    lib.ether_fcs.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    return lib


def ref_fcs(lib, b: bytes) -> int:
    v = lib.ether_fcs(b, len(b))
    assert v == zlib.crc32(b), "reference and zlib disagree"
    return v


# Edge lengths from SURVEY.md §4 plus the TX call-site range ends (70, 1514).
EDGE_LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 17, 31, 32, 33, 47, 48, 49, 59, 60, 61, 63, 64,
                65, 69, 70, 71, 95, 96, 97, 127, 128, 129, 255, 256, 257, 575, 576, 577, 1023,
                1024, 1025, 1487, 1488, 1489, 1513, 1514, 1515, 1516, 1517, 1518, 1519, 1535,
                1536, 1537, 1583, 1584, 1585, 3071, 3072, 3073, 4095, 4096, 4097, 8999, 9000,
                9001, 9018]


def main():
    lib = load_ref()
    rng = random.Random(20261015)

    # ---- known answers ----
    kat = {"source": "reference src/ether_fcs.c:4-19 compiled by oracle/Makefile (O2); zlib agrees",
           "cases": []}

    def add(name, data):
        kat["cases"].append({"name": name, "hex": data.hex() if len(data) <= 64 else None,
                             "fill": None, "len": len(data), "crc": ref_fcs(lib, data)})

    add("empty", b"")
    add("check_123456789", b"123456789")
    for n in (60, 1514, 1518, 9000):
        c = ref_fcs(lib, bytes(n))
        kat["cases"].append({"name": f"zeros_{n}", "hex": None, "fill": 0, "len": n, "crc": c})
        c = ref_fcs(lib, b"\xff" * n)
        kat["cases"].append({"name": f"ones_{n}", "hex": None, "fill": 255, "len": n, "crc": c})
    # residue property: fcs(data || LE32(fcs(data))) is the constant 0x2144DF1C
    res = set()
    for n in range(0, 80):
        d = bytes(rng.randrange(256) for _ in range(n))
        res.add(ref_fcs(lib, d + struct.pack("<I", ref_fcs(lib, d))))
    assert len(res) == 1
    kat["residue"] = res.pop()

    # ---- random frames at edge lengths, at every alignment 0..3, packed into one arena ----
    frames = []
    for n in EDGE_LENGTHS:
        for align in range(4):
            frames.append((n, align))
    for _ in range(200):  # plus random lengths 0..9018
        frames.append((rng.randrange(0, 9019), rng.randrange(4)))
    arena = bytearray()
    entries = []
    for n, align in frames:
        while len(arena) % 4 != align:
            arena.append(rng.randrange(256))
        off = len(arena)
        data = bytes(rng.randrange(256) for _ in range(n))
        arena += data
        entries.append({"off": off, "len": n, "crc": ref_fcs(lib, data)})
    arena += bytes(rng.randrange(256) for _ in range(5))
    with open(os.path.join(HERE, "vectors.bin"), "wb") as f:
        f.write(arena)

    # ---- SURVEY §8c dataset digest: xorshift64 seed 42, 1 M x 1518 B packed ----
    o = ctypes.CDLL(ORACLE_SO)
    nfr, L = 1 << 20, 1518
    buf = (ctypes.c_uint8 * (nfr * L))()
    st = ctypes.c_uint64(42)
    o.oracle_xorshift64_fill(buf, ctypes.c_size_t(nfr * L), ctypes.byref(st))
    addr = ctypes.addressof(buf)
    x = 0
    s = 0
    first = last = None
    for i in range(nfr):
        c = lib.ether_fcs(ctypes.c_void_p(addr + i * L), L)
        x ^= c
        s = (s + c) & ((1 << 64) - 1)
        if i == 0:
            first = c
        last = c
    digest = {"frames": nfr, "len": L, "seed": 42, "xor": x, "sum64": s, "first": first,
              "last": last, "first_bytes": bytes(buf[:4]).hex()}

    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump({"source": kat["source"], "arena": "vectors.bin", "frames": entries,
                   "xorshift_1m_1518": digest}, f, indent=0)
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kat, f, indent=1)
    print(f"{len(entries)} frames, arena {len(arena)} B; digest xor=0x{x:08X} sum=0x{s:016X}")


if __name__ == "__main__":
    sys.exit(main())
