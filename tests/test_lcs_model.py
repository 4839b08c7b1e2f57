"""The lane-chunk carry decomposition (tests/lcs_model.py) against zlib (= the reference ether_fcs,
/root/reference/src/ether_fcs.c:4-19): CPU only, small packed batches."""
import numpy as np
import pytest

from lcs_model import fcs_zlib, model_lcs


def _batch(lens, base, seed):
    rng = np.random.default_rng(seed)
    offs = base + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    total = int(offs[-1] + lens[-1])
    arena = rng.integers(0, 256, total, dtype=np.uint8).tobytes()
    return arena, [int(o) for o in offs], [int(x) for x in lens]


@pytest.mark.parametrize("G", [1, 2, 4])
@pytest.mark.parametrize("base", [0, 5, 16, 37])
def test_imix(G, base):
    rng = np.random.default_rng(G * 100 + base)
    lens = rng.choice(np.array([64] * 7 + [576] * 4 + [1518]), 90)
    arena, offs, lens = _batch(lens, base, base)
    got = model_lcs(arena, offs, lens, G=G, unit_frames=40)
    exp = [fcs_zlib(arena[o:o + n]) for o, n in zip(offs, lens)]
    assert got == exp


@pytest.mark.parametrize("G", [2, 4])
@pytest.mark.parametrize("L", [64, 65, 127, 128, 255, 256, 257, 511, 512, 1536])
def test_fixed_lengths(G, L):
    """Ends on and next to sub-chunk and lane-chunk edges (from base 0 every 64 B / 64 G B)."""
    arena, offs, lens = _batch(np.full(40, L), 0, L)
    got = model_lcs(arena, offs, lens, G=G, unit_frames=17)
    assert got == [fcs_zlib(arena[o:o + n]) for o, n in zip(offs, lens)]


@pytest.mark.parametrize("G", [2, 4])
def test_random_lengths(G):
    rng = np.random.default_rng(G)
    for trial in range(6):
        lens = rng.integers(64, 1537, 50)
        arena, offs, lens = _batch(lens, int(rng.integers(0, 64)), trial)
        got = model_lcs(arena, offs, lens, G=G, unit_frames=int(rng.integers(1, 50)))
        assert got == [fcs_zlib(arena[o:o + n]) for o, n in zip(offs, lens)]
