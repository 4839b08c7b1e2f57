"""N > 1 path on CPU: two ranks over gloo (127.0.0.1) run bench.py's sharding and timing logic.

The ranges come from the product's shard planner (fcs_shard_plan through bench.shard_range), for
fixed-length frames and for a byte-balanced IMIX batch.

Frames shard embarrassingly: each rank owns a contiguous slice of one global
counter-based frame stream, computes its CRCs (here with the oracle — test infrastructure; on
the GPU box the same ranges go to the HIP kernel), and the job reports all ranks' bytes over the
max rank time. Checks: the ranges partition the frame space; the gathered per-rank CRCs equal a
single-process pass over all frames (shard consistency); the MAX all-reduce and aggregate()
arithmetic; no collective touches frame data.
"""
import ctypes
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

TOTAL, L, SEED = 3001, 1518, 77
IMIX_BLK = 1200   # frames per GPU of the sharded IMIX bench config in these tests


def _oracle():
    o = ctypes.CDLL(os.path.join(ROOT, "oracle", "_build", "liboracle.so"))
    o.oracle_splitmix_fill.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
    o.oracle_fcs_fixed.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_size_t,
                                   ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    return o


def _crcs(o, lo, hi):
    n = hi - lo
    buf = np.empty(max(n, 1) * L, dtype=np.uint8)
    o.oracle_splitmix_fill(buf.ctypes.data, n * L, SEED, lo * L)
    out = np.zeros(max(n, 1), dtype=np.uint32)
    if n:
        o.oracle_fcs_fixed(buf.ctypes.data, L, L, n, out.ctypes.data, 1, 1)
    return out[:n]


def _imix(n):
    return np.random.default_rng(3).choice(np.array([64] * 7 + [576] * 4 + [1518], dtype=np.uint32), n)


def _crcs_var(o, ln, lo, hi):
    """CRCs of frames [lo, hi) of a packed IMIX stream (frame i at the prefix sum of ln)."""
    off = np.concatenate([[0], np.cumsum(ln, dtype=np.uint64)])
    buf = np.empty(int(off[-1]) + 8, dtype=np.uint8)
    o.oracle_splitmix_fill(buf.ctypes.data, int(off[-1]), SEED, 0)
    out = np.zeros(max(hi - lo, 1), dtype=np.uint32)
    o.oracle_fcs_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_int]
    if hi > lo:
        o_ = np.ascontiguousarray(off[lo:hi], dtype=np.uint64)
        l_ = np.ascontiguousarray(ln[lo:hi], dtype=np.uint32)
        o.oracle_fcs_batch(buf.ctypes.data, o_.ctypes.data, l_.ctypes.data, out.ctypes.data, hi - lo, 1)
    return out[:hi - lo]


def _worker(rank, world, port, q, mode="fixed"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    o = _oracle()
    if mode == "imix_bench":   # bench.py's configs[2] shard at N > 1 (imix_shard -> imix_sharded)
        lo, hi, ln, off, byte0, total = bench.imix_shard(world, rank, IMIX_BLK)
        buf = np.empty(total + 8, dtype=np.uint8)
        o.oracle_splitmix_fill(buf.ctypes.data, total, SEED, byte0)
        crc = np.zeros(hi - lo, dtype=np.uint32)
        o.oracle_fcs_batch.argtypes = [ctypes.c_void_p] * 4 + [ctypes.c_size_t, ctypes.c_int]
        o.oracle_fcs_batch(buf.ctypes.data, off.ctypes.data, ln.ctypes.data, crc.ctypes.data, hi - lo, 1)
        sizes = [None] * world
        dist.all_gather_object(sizes, (lo, hi, crc.tolist(), byte0, total))
        if rank == 0:
            q.put((sizes, 0.0))
        dist.destroy_process_group()
        return
    if mode == "host":   # bench.py's host-inclusive run at N > 1: synthetic run times, real gathering
        secs = [0.10 * (rank + 1), 0.30 * (rank + 1), 0.20 * (rank + 1)]
        allr, rep_max = bench.gather_host_times(torch, dist, world, rank, (rank + 1) << 30, secs, 0)
        if rank == 0:
            q.put((bench.host_aggregate(allr, rep_max), rep_max))
        dist.destroy_process_group()
        return
    if mode == "imix":
        ln = _imix(TOTAL)
        lo, hi = bench.shard_range(TOTAL, world, rank, ln)
    else:
        lo, hi = bench.shard_range(TOTAL, world, rank)
    dist.barrier()
    crc = _crcs_var(o, ln, lo, hi) if mode == "imix" else _crcs(o, lo, hi)
    elapsed = torch.tensor([0.5 + rank], dtype=torch.float64)   # synthetic per-rank times
    dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    sizes = [None] * world
    dist.all_gather_object(sizes, (lo, hi, crc.tolist()))
    dist.barrier()
    if rank == 0:
        q.put((sizes, float(elapsed.item())))
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world", [2, 4])
def test_two_rank_sharding_matches_single_pass(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    sizes, tmax = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # ranges partition [0, TOTAL) contiguously
    assert sizes[0][0] == 0 and sizes[-1][1] == TOTAL
    for a, b in zip(sizes, sizes[1:]):
        assert a[1] == b[0]
    gathered = np.concatenate([np.array(s[2], dtype=np.uint32) for s in sizes])
    assert np.array_equal(gathered, _crcs(_oracle(), 0, TOTAL))
    assert tmax == 0.5 + (world - 1)
    value, t = bench.aggregate([(s[1] - s[0]) * L for s in sizes], [0.5 + r for r in range(world)])
    assert t == 0.5 + (world - 1) and value == TOTAL * L / t


def test_two_rank_imix_byte_balanced_shards_match_single_pass():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "imix")) for r in range(world)]
    for p in procs:
        p.start()
    sizes, _ = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ln = _imix(TOTAL)
    assert sizes[0][0] == 0 and sizes[-1][1] == TOTAL and sizes[0][1] == sizes[1][0]
    b0, b1 = int(ln[:sizes[0][1]].sum()), int(ln[sizes[0][1]:].sum())
    assert abs(b0 - b1) <= 2 * 1518                      # byte-balanced cut from fcs_shard_plan
    gathered = np.concatenate([np.array(s[2], dtype=np.uint32) for s in sizes])
    assert np.array_equal(gathered, _crcs_var(_oracle(), ln, 0, TOTAL))


def test_shard_ranges_cover_eight_gpus():
    total = 512 << 20   # BASELINE configs[4]
    r = [bench.shard_range(total, 8, k) for k in range(8)]
    assert r[0][0] == 0 and r[-1][1] == total
    assert all(hi - lo == 64 << 20 for lo, hi in r)


@pytest.mark.parametrize("world", [2, 4])
def test_two_rank_imix_bench_path_shards_match_single_pass(world):
    """bench.py's N > 1 IMIX config (imix_shard): the global stream is `world` blocks of IMIX frames;
    the ranks' fcs_shard_plan ranges partition it, each rank's bytes start at its global byte
    position, and the gathered CRCs equal one pass over the whole stream (2 and 4 ranks)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "imix_bench")) for r in range(world)]
    for p in procs:
        p.start()
    sizes, _ = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    glob = np.tile(bench.imix_lengths(IMIX_BLK), world)
    assert sizes[0][0] == 0 and sizes[-1][1] == len(glob)
    for a, b in zip(sizes, sizes[1:]):
        assert a[1] == b[0]
    for s in sizes:   # each rank's bytes start at its global byte position
        assert s[3] == int(glob[:s[0]].sum())
    assert sum(s[4] for s in sizes) == int(glob.sum())
    gathered = np.concatenate([np.array(s[2], dtype=np.uint32) for s in sizes])
    assert np.array_equal(gathered, _crcs_var(_oracle(), glob, 0, len(glob)))


@pytest.mark.parametrize("world", [2, 4])
def test_host_inclusive_aggregate_over_ranks(world):
    """bench.py's host-inclusive run at N > 1: each rank's bytes and the median of
    its runs travel over gloo, the per-run maximum over ranks gives the aggregate: all ranks' bytes
    over the median of the slowest rank's run times. Rank r moves (r + 1) GiB in 0.1/0.3/0.2 x (r + 1) s."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, "host")) for r in range(world)]
    for p in procs:
        p.start()
    agg, rep_max = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert rep_max == pytest.approx([0.1 * world, 0.3 * world, 0.2 * world])
    total = sum((r + 1) << 30 for r in range(world))
    assert agg["bytes_all_ranks"] == total
    assert agg["secs_max_rank"] == pytest.approx(0.2 * world)
    assert agg["GB_s_aggregate"] == round(total / (0.2 * world) / 1e9, 2)
    assert [r["rank"] for r in agg["per_rank"]] == list(range(world))
    for r in agg["per_rank"]:   # each rank: its bytes over the median of its own runs
        assert r["secs"] == pytest.approx(0.2 * (r["rank"] + 1), abs=1e-4)
        assert r["GB_s"] == round(((r["rank"] + 1) << 30) / r["secs"] / 1e9, 2)
