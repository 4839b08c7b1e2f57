"""The product's shard planner (fcs_shard_plan; SURVEY.md §8e: contiguous frame ranges, split by a
byte-balanced prefix sum for variable lengths) against a Python restatement, on the CPU."""
import numpy as np
import pytest

import nstack_amd as na


def plan_ref(n, G, lengths=None):
    cut = [0] * (G + 1)
    cut[G] = n
    if lengths is None:
        for g in range(1, G):
            cut[g] = n * g // G
        return cut
    tot = int(sum(int(x) for x in lengths))
    acc, g = 0, 1
    for i in range(n):
        if g >= G:
            break
        acc += int(lengths[i])
        while g < G and acc * G >= tot * g:
            cut[g] = i + 1
            g += 1
    while g < G:
        cut[g] = n
        g += 1
    return cut


def imix(n, seed):
    return np.random.default_rng(seed).choice(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.uint32), n)


@pytest.mark.parametrize("G", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("n", [0, 1, 5, 1000, 100003])
def test_fixed_and_imix_plans_match_restatement(G, n):
    assert na.shard_plan(n, G) == plan_ref(n, G)
    ln = imix(n, n + G)
    cut = na.shard_plan(n, G, ln)
    assert cut == plan_ref(n, G, ln)
    assert cut[0] == 0 and cut[-1] == n and all(a <= b for a, b in zip(cut, cut[1:]))


@pytest.mark.parametrize("G", [2, 4, 8])
def test_imix_plan_is_byte_balanced(G):
    n = 1 << 20
    ln = imix(n, G)
    cut = na.shard_plan(n, G, ln)
    pre = np.concatenate([[0], np.cumsum(ln, dtype=np.uint64)])
    part = [int(pre[cut[g + 1]] - pre[cut[g]]) for g in range(G)]
    assert max(part) - min(part) <= 2 * 1518          # within a couple of frames of equal bytes


def test_edge_cases():
    assert na.shard_plan(10, 4, np.zeros(10, dtype=np.uint32)) == plan_ref(10, 4, [0] * 10)
    big = np.full(7, 0xFFFFFFFF, dtype=np.uint32)        # 64-bit prefix, 128-bit products
    assert na.shard_plan(7, 8, big) == plan_ref(7, 8, big)
    with pytest.raises(na.FcsError):
        na.shard_plan(10, 0)
