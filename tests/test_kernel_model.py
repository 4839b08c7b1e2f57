"""CPU replay of the kernel's arithmetic (tests/kernel_model.py) against the golden fixtures.

Validates the constant tables the product library builds (fcs_tables_blob), the v_perm LDS
addressing, front-lane init/masking, segment jumps and lane shifts — without a GPU."""
import random
import zlib

import pytest

import kernel_model as km  # noqa: E402

na = pytest.importorskip("nstack_amd")


@pytest.fixture(scope="module")
def lds():
    return km.build_lds(na.tables_blob())


def test_blob_slice_tables_match_reference_polynomial(lds):
    blob = na.tables_blob()
    # T0 is the byte-wise table of the reflected polynomial 0xEDB88320
    for b in (0, 1, 128, 255):
        r = b
        for _ in range(8):
            r = (r >> 1) ^ (0xEDB88320 if r & 1 else 0)
        assert blob[b] == r


def test_model_on_golden_vectors(lds, golden):
    arena = golden["arena"]
    frames = golden["vectors"]["frames"]
    for fr in frames[::3]:
        assert km.model_frame(lds, arena, fr["off"], fr["len"]) == fr["crc"], fr


def test_model_edges_and_alignment(lds):
    rng = random.Random(9)
    mem = bytes(rng.randrange(256) for _ in range(12000))
    for L in (0, 1, 3, 4, 47, 48, 49, 70, 1488, 1489, 1514, 1518, 1536, 1537, 3073, 9000):
        for S in (0, 1, 2, 3, 12000 - L):
            if 0 <= S and S + L <= len(mem):
                assert km.model_frame(lds, mem, S, L) == zlib.crc32(mem[S:S + L]), (L, S)


def _shift(s, n):
    """A_n: the CRC register advanced over n zero bytes (reflected 0xEDB88320)."""
    for _ in range(n):
        for _ in range(8):
            s = (s >> 1) ^ (0xEDB88320 if s & 1 else 0)
    return s


def test_flat_kernel_chunk_shift_tables():
    """The flat variable-length kernel's C_c = A_{96c} nibble tables (fcs_tables.hpp kBlobFlat,
    136-dword stride per c): chunk_shift(s, c) = XOR_t C_c[t][nibble_t(s)] must equal A_{96c}(s)."""
    blob = na.tables_blob()
    flat = km.BLOB_INV + km.CHUNK + 8 * 16   # kBlobM768 + 8 * 16
    rng = random.Random(4)
    for c in (0, 1, 5, 15):
        for _ in range(3):
            s = rng.getrandbits(32)
            v = 0
            for t in range(8):
                v ^= int(blob[flat + c * 136 + t * 16 + ((s >> (4 * t)) & 15)])
            assert v == _shift(s, 96 * c), (c, hex(s))
