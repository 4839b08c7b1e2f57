"""Generate the Internet-checksum fixtures (tests/golden/inet_vectors.{bin,json}).

    python tests/golden/make_inet_golden.py

The reference's src/ip.c could not be built here (DESIGN.md §2 records the refusal), so the
expected values come from an INDEPENDENT formulation written only for this script: RFC 1071
over big-endian 16-bit words with a zero pad byte, the pseudo headers of RFC 793 / RFC 768, and
the two nstack-specific rules read from the reference source:
  * ip_checksum / tcp_checksum start the accumulator at 0xffff (src/ip.c:42, src/tcp.c:172),
    which only matters when every summed word is zero: they return 0x0000 where RFC 1071's
    zero-initialised sum returns 0xffff;
  * the 16-bit length in both pseudo headers is htons() of a size_t, i.e. len mod 65536
    (src/tcp.c:187, src/udp.c:167); the UDP addresses are the raw in_addr_t values the caller
    passes (src/udp.c:143,160-164), the TCP ones are htonl() of host-order addresses (:185-186).
The functions return the checksum as a host-order uint16 whose memory bytes are the on-wire
bytes, so the little-endian value recorded here is the byte swap of the big-endian checksum.
The oracle (oracle/inet_oracle.c, a loop-for-loop restatement of the reference) is checked
against these vectors by tests/test_inet_oracle.py; the GPU kernel by tests/test_gpu_inet.py.
"""
import json
import os
import random
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
MODES = {"ip": 0, "tcp": 1, "udp": 2}


def be_sum(b: bytes) -> int:
    if len(b) & 1:
        b = b + b"\x00"
    return sum(struct.unpack(f">{len(b) // 2}H", b)) if b else 0


def fold(s: int) -> int:
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def swap16(x: int) -> int:
    return ((x & 0xFF) << 8) | (x >> 8)


def witness(mode: str, data: bytes, src: int = 0, dst: int = 0) -> int:
    """Expected return value (host-order u16 on a little-endian host)."""
    L = len(data) & 0xFFFF
    if mode == "ip":
        s = be_sum(data)
    elif mode == "tcp":
        s = be_sum(struct.pack(">IIBBH", src, dst, 0, 6, L)) + be_sum(data)
    else:  # udp: the raw in_addr_t bytes as they lie in (little-endian) memory
        s = be_sum(struct.pack("<II", src, dst)) + 17 + L + be_sum(data)
    if s == 0 and mode in ("ip", "tcp"):
        return 0x0000          # acc = 0xffff never folds away: ~0xffff
    return swap16(~fold(s) & 0xFFFF)


EDGE = [0, 1, 2, 3, 4, 5, 6, 7, 8, 15, 16, 17, 19, 20, 21, 31, 32, 33, 40, 59, 60, 61, 63, 64, 65,
        127, 128, 129, 255, 256, 257, 575, 576, 577, 1023, 1024, 1025, 1479, 1480, 1481, 1499, 1500,
        1501, 1513, 1514, 1517, 1518, 1519, 2047, 2048, 4095, 4096, 8999, 9000, 65535, 65536, 65537]


def main():
    rng = random.Random(0x1CE7)
    arena = bytearray()
    recs = []

    def add(mode, data, src=0, dst=0, tag=""):
        pad = rng.randrange(0, 16)            # every start alignment mod 16
        arena.extend(rng.randbytes(pad))
        off = len(arena)
        arena.extend(data)
        recs.append({"mode": mode, "off": off, "len": len(data), "src": src, "dst": dst,
                     "expect": witness(mode, bytes(data), src, dst), "tag": tag})

    for L in EDGE:
        for mode in MODES:
            add(mode, rng.randbytes(L), rng.getrandbits(32), rng.getrandbits(32), f"edge{L}")
    for L in (0, 1, 2, 20, 21, 1500):
        for mode in MODES:
            add(mode, bytes(L), 0, 0, f"zeros{L}")
            add(mode, b"\xff" * L, rng.getrandbits(32), rng.getrandbits(32), f"ones{L}")
    # the UDP loop's "if (sum & 0x80000000)" fold (src/udp.c:150-151) needs > 32768 words of 0xffff
    add("udp", b"\xff" * 131072, 0xFFFFFFFF, 0xFFFFFFFF, "udp_inner_fold")
    add("ip", b"\xff" * 131073, 0, 0, "ip_big_odd")
    for _ in range(300):
        L = rng.choice([rng.randrange(0, 64), rng.randrange(0, 1600), rng.randrange(1600, 10000)])
        mode = rng.choice(list(MODES))
        add(mode, rng.randbytes(L), rng.getrandbits(32), rng.getrandbits(32), "rand")
    # headers whose checksum field is already filled in: ip_checksum over them must return 0
    for _ in range(20):
        h = bytearray(rng.randbytes(20))
        h[0] = 0x45
        h[10:12] = b"\x00\x00"
        c = witness("ip", bytes(h))
        h[10:12] = struct.pack("<H", c)
        add("ip", bytes(h), tag="ip_hdr_filled")
    arena.extend(rng.randbytes(16))

    kat = [
        # RFC 1071 §3 numeric example: words 0001 f203 f4f5 f6f7, sum ddf2, checksum 220d on the wire
        {"mode": "ip", "hex": "0001f203f4f5f6f7", "expect_wire": "220d"},
        # textbook IPv4 header (checksum field zeroed): on-wire checksum b861
        {"mode": "ip", "hex": "450000730000400040110000c0a80001c0a800c7", "expect_wire": "b861"},
        # the same header with its checksum in place verifies to 0
        {"mode": "ip", "hex": "450000730000400040110b861c0a80001c0a800c7".replace("0b861", "b861"),
         "expect_wire": "0000"},
        # all-zero data: nstack's acc = 0xffff start returns 0 (RFC 1071 zero-start would give ffff)
        {"mode": "ip", "hex": "0000000000000000", "expect_wire": "0000"},
        {"mode": "ip", "hex": "", "expect_wire": "0000"},
    ]
    for k in kat:
        got = witness(k["mode"], bytes.fromhex(k["hex"]))
        assert struct.pack("<H", got).hex() == k["expect_wire"], (k, hex(got))

    with open(os.path.join(HERE, "inet_vectors.bin"), "wb") as f:
        f.write(bytes(arena))
    with open(os.path.join(HERE, "inet_vectors.json"), "w") as f:
        json.dump({"arena": "inet_vectors.bin", "modes": MODES, "packets": recs, "kat": kat,
                   "generator": "tests/golden/make_inet_golden.py (independent RFC 1071 witness)"},
                  f, indent=0)
    print(f"{len(recs)} packets, {len(arena)} arena bytes")


if __name__ == "__main__":
    main()
