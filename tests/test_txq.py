"""Batched TX call site (include/nstack_txq.h) — host logic that needs no GPU.

ether_send (src/linux/ether.c:214-272) rejects frame_size > 1518 with -EMSGSIZE before touching
anything (:234-237); frame_size = 14 + max(bsize, 56) + 4 (:222-224). Without a GPU the queue
must fail every frame with -ENODEV and send nothing (no unchecked FCS leaves).
"""
import os
import socket
import threading

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


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU error path")
def test_no_gpu_fails_every_frame_and_sends_nothing():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    b.setblocking(False)
    res = []
    with na.TxQueue(MAC, a.fileno(), max_batch=4, flush_usec=50) as q:
        th = [threading.Thread(target=lambda k=k: res.append(q.send(DST, 0x0806, bytes([k]) * (10 * k))))
              for k in range(10)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        q.flush()
        frames, batches, errors = q.stats()
        why = q.last_error()
    assert res == [-19] * 10                                     # -ENODEV for every caller
    assert why                                                   # the failing step's reason
    assert frames == 10 and batches >= 3 and errors == 10       # batches of at most 4
    with pytest.raises(BlockingIOError):
        b.recv(2048)
    a.close(), b.close()


@pytest.mark.timeout(120)
@pytest.mark.skipif(_gpu_visible(), reason="checks the queue machinery on the no-GPU error path")
@pytest.mark.parametrize("max_batch,linger", [(1, 0), (8, 0), (64, 20), (4096, 2000)])
def test_many_producers_no_lost_frames(max_batch, linger):
    """Lock-free slot reservation under contention: sync and fire-and-forget producers together,
    tiny and large batches, spinning and sleeping lingers. Every frame is accounted for once and
    every sync caller gets its (here -ENODEV) result; flush() and close() return."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    res = []
    lock = threading.Lock()
    n_sync, n_async, per = 12, 4, 150
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
    total = (n_sync + n_async) * per
    assert res == [-19] * (n_sync * per)
    assert frames == total and errors == total
    assert batches >= -(-total // max_batch)
    a.close(), b.close()
