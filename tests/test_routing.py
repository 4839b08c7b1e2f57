"""Which kernel a fixed-length batch takes (CPU; host arithmetic only, no device call).

fcs_debug_fixed_route (include/nstack_fcs.h) names the kernel ether_fcs_fixed_dev would launch for
a batch: the same predicates as launch_fixed and fcs::launch_fcs (fcs_launch.hpp). The table below
is the round-4 band map (DESIGN.md §3.2d band map, §3.3c, §4.2b): packed batches of 1 M frames, the
bank rule's exceptions, strides the slot kernels do not take, and small batches (at or below the
16384-frame threshold the short and flat routes do not apply).
"""
import os
import sys

import pytest

import nstack_amd as na

BASE = 1 << 30
BIG = 1 << 20

PACKED = {
    32: "short:16", 60: "short:16", 64: "short:16", 74: "short:24", 96: "short:24", 100: "short:32",
    128: "short:32", 129: "flat", 130: "wide4:9", 200: "wide4:14", 256: "flat", 300: "wide4:20",
    320: "flat", 400: "wide8:14", 512: "flat", 576: "wide8:19", 640: "flat", 700: "wide8:23", 768: "flat",
    868: "wide8:28", 869: "flat", 870: "wide16:15", 1000: "wide16:18", 1157: "wide16:20", 1476: "wide16:24",
    1477: "wide16:26", 1495: "wide16:26", 1496: "lds-dma", 1518: "lds-dma", 1524: "lds-dma", 1525: "wide16:26",
    1536: "wide16:26", 1604: "wide16:26", 1605: "wide16:30", 1787: "wide16:30", 1788: "wide16:32",
    1988: "wide16:32", 2500: "segment:22", 3049: "segment:26", 3073: "segment:26", 9000: "segment:30", 9216: "segment:30",
    65536: "segment:32",
}


@pytest.fixture(scope="module")
def lib():
    na.load()
    return na


@pytest.mark.parametrize("L", sorted(PACKED))
def test_packed_route(lib, L):
    assert lib.fixed_route(BASE, L, L, BIG) == PACKED[L]


@pytest.mark.parametrize("L,stride,want", [
    (1518, 2048, "single"),      # 3 stride + len > 6126: no LDS-DMA slot
    (500, 2000, "flat"),         # eight 2000-B strides do not fit a 7 KiB slot
    (1000, 2049, "flat"),        # mid-length widths take strides up to 2048
    (1600, 1700, "wide16:26"),   # 3 * 1700 + 1600 <= 7150
    (1600, 1851, "wide16:32"),   # one past the 7 KiB slot: the 128-B windows, 8 KiB slots
    (64, 4096, "short:16"),      # the short-frame kernel takes any stride
    (0, 4, "flat"),              # empty frames
])
def test_strided_route(lib, L, stride, want):
    assert lib.fixed_route(BASE, stride, L, BIG) == want


def test_small_batches(lib):
    """At or below the small-batch threshold the short and flat routes do not apply: short frames
    take the quarter-wave kernels, the slot kernels still take what their slots fit."""
    assert lib.fixed_route(BASE, 64, 64, 16384) == "generic"
    assert lib.fixed_route(BASE, 64, 64, 16385) == "short:16"
    assert lib.fixed_route(BASE, 1518, 1518, 100) == "lds-dma"
    assert lib.fixed_route(BASE, 1518, 1518, 2) == "single"   # an arena of less than two LDS-DMA slots
    assert lib.fixed_route(BASE, 100, 100, 1) == "tiny"       # under two 96-B chunks of bytes
    assert lib.fixed_route(BASE, 1518, 1518, 0) == "none"


def test_sweep_tool_agrees(lib):
    """tools/len_sweep.py's restatement of the choice names the same family for packed lengths
    (the 4- and 8-lane families name their bank-rule exception)."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import len_sweep
    prefix = {"short": "short", "flat": "flat", "wide4": "wide, 4 lanes", "wide8": "wide, 8 lanes",
              "segment": "segment", "lds-dma": "lds-dma", "generic": "generic"}
    for L in sorted(PACKED):
        got = lib.fixed_route(BASE, L, L, BIG)
        fam = len_sweep.family(L)
        kind = got.split(":")[0]
        if kind == "flat" and "bank-phased" in fam:
            continue
        if kind == "wide16":
            assert fam.startswith("wide") and "lanes" not in fam, (L, got, fam)
        else:
            assert fam.startswith(prefix[kind]), (L, got, fam)


def _seg_item_words():
    import re
    hdr = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nstack_amd", "csrc", "fcs_launch.hpp")
    return int(re.search(r"#define FCS_SEG_ITEM_WORDS (\d+)", open(hdr).read()).group(1))


def test_segment_width_rule(lib):
    """Packed batches the segment route takes pick the segment width with the least per-lane work,
    m (WD + K) for m = ceil(len / cover) (fcs_launch.hpp segment_wd: cover 1524 B for WD 24, the
    wide kernel's 15 (4 WD - 4) + 4 WD for the other widths; ties keep the earlier candidate)."""
    K = _seg_item_words()
    order = [24, 15, 16, 18, 19, 20, 22, 23, 26, 30, 32]   # candidates in the order segment_wd tries them
    cover = {w: 15 * (4 * w - 4) + 4 * w for w in order}
    cover[24] = 1524
    seen = set()
    for L in list(range(1950, 12000, 7)) + [16384, 40000, 65536, 100000]:
        got = lib.fixed_route(BASE, L, L, BIG)
        if not got.startswith("segment"):
            continue
        costs = [-(-L // cover[w]) * (w + K) for w in order]
        best = order[costs.index(min(costs))]   # the first candidate at the least cost
        assert got == ("segment" if best == 24 else f"segment:{best}"), (L, got, best)
        seen.add(best)
    assert {24, 26, 30, 32} <= seen
