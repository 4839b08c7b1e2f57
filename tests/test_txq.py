"""Batched TX call site (include/nstack_txq.h) — host logic that needs no GPU.

ether_send (src/linux/ether.c:214-272) rejects frame_size > 1518 with -EMSGSIZE before touching
anything (:234-237); frame_size = 14 + max(bsize, 56) + 4 (:222-224), and it never fails for FCS
reasons. Without a GPU the queue's GPU step fails, so every batch's FCSs come from the library's
host CRC: each frame must still leave byte-identical to ether_send's (checked against
the oracle's restatement of src/ether_fcs.c), each caller gets frame_size, and the fallback is counted.
"""
import os
import socket
import struct
import threading
from collections import Counter

import pytest

import nstack_amd as na

MAC = bytes([2, 0, 0, 0, 0, 1])
DST = bytes([2, 0, 0, 0, 0, 2])


def _gpu_visible():
    return os.path.exists("/dev/kfd")


def test_emsgsize_rule_matches_ether_send():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    with na.TxQueue(MAC, a.fileno(), max_batch=8, flush_usec=100) as q:
        assert q.send(DST, 0x0800, b"x" * 1501) == -90          # -EMSGSIZE: 14+1501+4 > 1518
        assert q.send(DST, 0x0800, b"x" * 5000) == -90
        assert q.stats() == (0, 0, 0)                            # nothing was queued
    a.close(), b.close()


def test_bad_arguments():
    lib = na.load()
    assert lib.fcs_txq_create(None, 8, 10, None, None) is None
    assert lib.fcs_txq_send(None, DST, 0x0800, b"", 0) == -22
    assert lib.fcs_txq_flush(None) == -22


def ether_send_frame(oracle, dst, proto, payload):
    frame_size = 14 + max(len(payload), 56) + 4                 # :222-224
    f = dst + MAC + struct.pack(">H", proto) + payload          # :257-260
    f += b"\0" * (frame_size - 4 - len(f))                      # :261
    return f + struct.pack("<I", oracle.oracle_ether_fcs(f, len(f)))   # :262-263


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU path")
def test_no_gpu_host_crc_sends_every_frame(oracle):
    """The GPU step fails (no GPU): the host CRC answers, the frames leave as ether_send builds them."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    b.setblocking(False)
    res = []
    plans = [(bytes([k]) * 6, 0x0806 + k, bytes([k]) * (10 * k + (k % 3) * 500)) for k in range(10)]
    with na.TxQueue(MAC, a.fileno(), max_batch=4, flush_usec=50, gpu_only=True) as q:   # every batch to the GPU
        th = [threading.Thread(target=lambda p=p: res.append((q.send(*p), 14 + max(len(p[2]), 56) + 4)))
              for p in plans]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        frames, batches, errors = q.stats()
        host_batches, host_frames = q.fallbacks()
        why = q.last_error()
    assert all(r == want for r, want in res) and len(res) == 10   # frame_size for every caller
    assert why                                                   # the failing GPU step's reason
    assert frames == 10 and batches >= 3 and errors == 0        # batches of at most 4
    assert host_batches == batches and host_frames == 10
    assert na.engine_stats()["host_batches"] >= host_batches
    got = [b.recv(2048) for _ in range(10)]
    with pytest.raises(BlockingIOError):
        b.recv(2048)
    assert Counter(got) == Counter(ether_send_frame(oracle, *p) for p in plans)
    a.close(), b.close()


@pytest.mark.timeout(120)
@pytest.mark.skipif(_gpu_visible(), reason="checks the queue machinery on the no-GPU (host CRC) path")
@pytest.mark.parametrize("max_batch,linger", [(1, 0), (8, 0), (64, 20), (4096, 2000)])
def test_many_producers_no_lost_frames(max_batch, linger):
    """Lock-free slot reservation under contention: sync and fire-and-forget producers together,
    tiny and large batches, spinning and sleeping lingers. Every frame is accounted for once and
    every sync caller gets its result (frame_size, from the host CRC here); flush() and close()
    return."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    res = []
    lock = threading.Lock()
    n_sync, n_async, per = 12, 4, 150
    total = (n_sync + n_async) * per
    received = []
    drain = threading.Thread(target=lambda: received.extend(b.recv(2048) for _ in range(total)))
    drain.start()   # the frames now leave (host CRC): keep the socket from filling up
    with na.TxQueue(MAC, a.fileno(), max_batch=max_batch, flush_usec=linger) as q:
        def sync_worker(k):
            mine = [q.send(DST, 0x0800, bytes([k]) * (k * 37 % 1400)) for _ in range(per)]
            with lock:
                res.extend(mine)

        def async_worker(k):
            for i in range(per):
                assert q.send_async(DST, 0x0800, bytes([i & 255]) * (i % 300)) > 0

        th = [threading.Thread(target=sync_worker, args=(k,)) for k in range(n_sync)]
        th += [threading.Thread(target=async_worker, args=(k,)) for k in range(n_async)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        frames, batches, errors = q.stats()
    drain.join(timeout=60)
    assert len(received) == total
    assert sorted(res) == sorted(14 + max(k * 37 % 1400, 56) + 4 for k in range(n_sync) for _ in range(per))
    assert frames == total and errors == 0
    assert batches >= -(-total // max_batch)
    a.close(), b.close()


@pytest.mark.parametrize("gpu_only", [False, True])
def test_sync_callers_send_their_own_frames(oracle, gpu_only):
    """fcs_txq_send with nothing of the caller's own queued sends the frame itself (ether_send's body
    with the library's host CRC, the sink called with a batch of one): counted as host-CRC batches by
    design, no GPU step, no failure answer; so this runs the same with or without a GPU. gpu_only
    (fcs_txq_set_sync_host off, host_max 0) sends every frame through a batch's GPU step instead
    (here, without a GPU, answered by the host CRC after the failure and counted as such)."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    b.setblocking(False)
    plans = [(bytes([k]) * 6, 0x0800, bytes([k]) * (k * 150 % 1501)) for k in range(24)]
    with na.TxQueue(MAC, a.fileno(), max_batch=8, flush_usec=0, gpu_only=gpu_only) as q:
        res = [q.send(*p) for p in plans]
        q.flush()
        frames, batches, errors = q.stats()
        small_batches, small_frames, gpu_batches = q.paths()
        host_batches, host_frames = q.fallbacks()
    assert res == [14 + max(len(p[2]), 56) + 4 for p in plans]
    assert frames == 24 and errors == 0
    if not gpu_only:
        assert (small_batches, small_frames, batches) == (24, 24, 24) and host_batches == 0 and gpu_batches == 0
    else:
        assert small_batches == 0 and small_frames == 0
        if not _gpu_visible():
            assert (host_batches, host_frames) == (batches, 24)
    got = [b.recv(2048) for _ in range(24)]
    assert Counter(got) == Counter(ether_send_frame(oracle, *p) for p in plans)
    a.close(), b.close()


@pytest.mark.parametrize("host_max,expect_small", [(None, None), (1 << 30, True), (0, False)])
def test_async_batches_below_the_gpu_minimum_take_the_host_crc(oracle, host_max, expect_small):
    """Fire-and-forget batches whose covered bytes total at most the GPU minimum
    (fcs_txq_set_host_max, default 16 KiB) are computed by the flusher with the host CRC: counted as
    small batches, not as failure answers. host_max 0 sends every batch to the GPU step (here, without
    a GPU, answered by the host CRC after the failure)."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    b.setblocking(False)
    plans = [(bytes([k]) * 6, 0x0806, bytes([k]) * (k * 150 % 1501)) for k in range(40)]
    with na.TxQueue(MAC, a.fileno(), max_batch=8, flush_usec=0, host_max=host_max) as q:
        if host_max is None:
            assert q.set_host_max(16384) == 16384   # the documented default
        res = [q.send_async(*p) for p in plans]
        q.flush()
        frames, batches, errors = q.stats()
        small_batches, small_frames, gpu_batches = q.paths()
        host_batches, host_frames = q.fallbacks()
    assert res == [14 + max(len(p[2]), 56) + 4 for p in plans]
    assert frames == 40 and errors == 0
    assert small_batches + gpu_batches + host_batches == batches
    if expect_small:
        assert (small_batches, small_frames) == (batches, 40) and host_batches == 0 and gpu_batches == 0
    elif expect_small is False:
        assert small_batches == 0 and small_frames == 0
        if not _gpu_visible():
            assert (host_batches, host_frames) == (batches, 40)
    got = [b.recv(2048) for _ in range(40)]
    assert Counter(got) == Counter(ether_send_frame(oracle, *p) for p in plans)
    a.close(), b.close()


@pytest.mark.timeout(120)
@pytest.mark.parametrize("max_batch", [64, 512])
def test_per_thread_order_kept(max_batch):
    """Every producer's frames leave in the order it queued them, across shards and batches (the
    per-thread floor of enqueue; tools/tsan/run.sh drives the same check with C threads). Host CRC
    by design here (fire-and-forget batches below the GPU minimum), so no GPU is needed."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    P, per = 6, 1500
    total = P * per
    got = []
    drain = threading.Thread(target=lambda: got.extend(b.recv(2048) for _ in range(total)))
    drain.start()
    with na.TxQueue(MAC, a.fileno(), max_batch=max_batch, flush_usec=0, host_max=1 << 40) as q:
        def producer(t):
            for i in range(per):
                assert q.send_async(DST, 0x0806, bytes([t]) + i.to_bytes(4, "little") + bytes(i % 90)) > 0
        th = [threading.Thread(target=producer, args=(t,)) for t in range(P)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        q.flush()
    drain.join(timeout=60)
    a.close(), b.close()
    assert len(got) == total
    last = [-1] * P
    for f in got:
        t, i = f[14], int.from_bytes(f[15:19], "little")
        assert i > last[t], (t, i, last[t])
        last[t] = i
