"""The multi-device host path on a one-GPU box (fcs_engine.cpp run_host_sharded).

The host entry points shard a batch over the engine's devices: byte-balanced cuts from
fcs_shard_plan, one host thread and one chunked pipeline (streams, pinned staging, events) per
device, results written back in place. With NSTACK_FCS_ALIAS_DEVICES=1 (a test hook)
fcs_engine_init(k) accepts k devices beyond the HIP device count; engine device d >= count gets a
state of its own on HIP device d mod count. So fcs_engine_init(3) on one GPU runs three shards on
three threads with three independent pipelines. Every result is checked against zlib.crc32 (the
stdlib CRC-32, equal to src/ether_fcs.c:4-19), for the fixed, variable-length, TX and RX-verify
host entry points.
"""
import struct
import zlib

import numpy as np
import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def three_devices():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    na.load()
    os.environ["NSTACK_FCS_ALIAS_DEVICES"] = "1"
    try:
        assert na.engine_init(3) == 3
        assert na.load().fcs_engine_device_count() == 3
        yield 3
    finally:
        del os.environ["NSTACK_FCS_ALIAS_DEVICES"]
        na.engine_init(0)   # back to the real devices


def crcs(buf, offs, lens):
    return np.array([zlib.crc32(buf[int(o):int(o) + int(l)].tobytes()) for o, l in zip(offs, lens)], dtype=np.uint32)


def test_fixed_host_three_shards(three_devices):
    L, n = 1518, 9001   # G = min(3, n / 1024) = 3
    host = np.random.default_rng(1).integers(0, 256, n * L, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint32)
    before = na.engine_host_stats()
    na.fixed_host(host, L, L, n, out)
    after = na.engine_host_stats()
    assert np.array_equal(out, crcs(host, np.arange(n) * L, np.full(n, L)))
    assert after["sharded_calls"] - before["sharded_calls"] == 1
    assert after["shard_jobs"] - before["shard_jobs"] == 3


def test_batch_host_three_shards_byte_balanced(three_devices):
    rng = np.random.default_rng(2)
    n = 20011
    ln = rng.choice(np.array([64] * 7 + [576] * 4 + [1518] + [0, 9000], dtype=np.uint32), n)
    off = np.zeros(n, dtype=np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    total = int(off[-1]) + int(ln[-1])
    arena = rng.integers(0, 256, total + 8, dtype=np.uint8)
    out = np.zeros(n, dtype=np.uint32)
    na.batch_host(arena, total, off, ln, out, n)
    assert np.array_equal(out, crcs(arena, off, ln))
    cut = na.shard_plan(n, 3, ln)
    assert len(cut) == 4 and cut[0] == 0 and cut[-1] == n and all(a < b for a, b in zip(cut, cut[1:]))


def test_tx_host_three_shards(three_devices):
    rng = np.random.default_rng(3)
    stride, n = 1536, 6007
    cov = rng.integers(70, 1515, n).astype(np.uint32)
    arena = rng.integers(0, 256, n * stride, dtype=np.uint8)
    exp = arena.copy()
    for i in range(n):
        c = zlib.crc32(exp[i * stride:i * stride + int(cov[i])].tobytes())
        exp[i * stride + int(cov[i]):i * stride + int(cov[i]) + 4] = np.frombuffer(struct.pack("<I", c), dtype=np.uint8)
    na.tx_host(arena, stride, cov, n)
    assert np.array_equal(arena, exp)


def test_verify_host_three_shards(three_devices):
    rng = np.random.default_rng(4)
    n, L = 4099, 1518
    host = rng.integers(0, 256, n * L, dtype=np.uint8)
    for i in range(n):
        host[i * L + L - 4:i * L + L] = np.frombuffer(struct.pack("<I", zlib.crc32(host[i * L:i * L + L - 4].tobytes())),
                                                      dtype=np.uint8)
    bad_idx = sorted(set(int(x) for x in rng.integers(0, n, 17)) | {0, n - 1})
    for i in bad_idx:
        host[i * L + int(rng.integers(0, L))] ^= np.uint8(0x10)
    off = (np.arange(n) * L).astype(np.uint64)
    ln = np.full(n, L, dtype=np.uint32)
    ok = np.zeros(n, dtype=np.uint8)
    nbad = na.verify_host(host, n * L, off, ln, ok, n)
    exp = np.ones(n, dtype=np.uint8)
    exp[bad_idx] = 0
    assert nbad == len(bad_idx)
    assert np.array_equal(ok, exp)
