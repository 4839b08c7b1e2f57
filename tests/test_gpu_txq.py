"""Batched TX call site on the GPU: byte-identical frames to ether_send, per-call return values.

Expected frames are built from ether_send's own layout (src/linux/ether.c:222-263): dst, src MAC,
htons(proto), payload, zero pad, then LE32 of ether_fcs over the covered bytes — the FCS from the
oracle's restatement of src/ether_fcs.c. Many producer threads send concurrently through one
queue; the receiving end of a socketpair must see exactly the expected multiset of frames.
"""
import random
import socket
import struct
import threading
from collections import Counter

import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

MAC = bytes([0x02, 0x42, 0xAC, 0x11, 0x00, 0x02])


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    na.load()
    return torch.device("cuda:0")


def ether_send_frame(oracle, dst, proto, payload):
    frame_size = 14 + max(len(payload), 56) + 4                 # :222-224
    f = dst + MAC + struct.pack(">H", proto) + payload          # :257-260
    f += b"\0" * (frame_size - 4 - len(f))                      # :261
    return f + struct.pack("<I", oracle.oracle_ether_fcs(f, len(f)))   # :262-263


@pytest.mark.parametrize("gpu_only", [True, False])   # every frame through a GPU step / the defaults
@pytest.mark.parametrize("max_batch,flush_usec", [(1, 0), (64, 200), (1024, 2000)])
def test_concurrent_producers_byte_identical(dev, oracle, max_batch, flush_usec, gpu_only):
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    P, M = 8, 300
    plans = []
    for t in range(P):
        r = random.Random(1000 * max_batch + t)
        plans.append([(bytes(r.randrange(256) for _ in range(6)), r.choice([0x0800, 0x0806, 0x86DD]),
                       bytes(r.randrange(256) for _ in range(r.choice([0, 1, 55, 56, 57, r.randrange(0, 1501), 1500]))))
                      for _ in range(M)])
    expect = Counter(ether_send_frame(oracle, *x) for p in plans for x in p)
    got, results = [], [[] for _ in range(P)]
    total = P * M

    def reader():
        while len(got) < total:
            got.append(b.recv(2048))

    rd = threading.Thread(target=reader)
    rd.start()
    with na.TxQueue(MAC, a.fileno(), max_batch=max_batch, flush_usec=flush_usec, gpu_only=gpu_only) as q:
        def producer(t):
            for dst, proto, payload in plans[t]:
                results[t].append((q.send(dst, proto, payload), 14 + max(len(payload), 56) + 4))
        th = [threading.Thread(target=producer, args=(t,)) for t in range(P)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        q.flush()
        frames, batches, errors = q.stats()
        small_batches, small_frames, gpu_batches = q.paths()
        assert q.fallbacks() == (0, 0)                           # no GPU step failed
        assert small_batches + gpu_batches == batches
        if gpu_only:
            assert gpu_batches == batches                        # every batch's FCSs came from the GPU
            if max_batch == 1:
                assert batches == total
    rd.join(timeout=60)
    a.close(), b.close()
    assert all(r == want for rs in results for r, want in rs)   # per-call return = frame_size
    assert frames == total and 1 <= batches <= total and errors == 0
    assert Counter(got) == expect
    for f in got:                                                # every frame carries a valid FCS
        assert oracle.oracle_ether_fcs(f, len(f)) == 0x2144DF1C


def test_batches_above_the_gpu_minimum_run_the_kernel(dev, oracle):
    """The GPU minimum (fcs_txq_set_host_max) splits the batches: every batch of more covered bytes
    than it ran the GPU step (counted as a GPU batch, none answered by the host CRC after a failure),
    every batch at or below it was computed by the host CRC by design. Fire-and-forget producers
    with 1500-B payloads (1514 covered bytes) fill batches of up to 64 frames; the minimum is 16 such
    frames, so both kinds occur; every frame leaves exact."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    P, M = 4, 600
    payload = [bytes((t * 7 + i) & 255 for i in range(1500)) for t in range(P)]
    total = P * M
    got = []
    rd = threading.Thread(target=lambda: got.extend(b.recv(2048) for _ in range(total)))
    rd.start()
    h0 = na.engine_stats()["host_batches"]
    with na.TxQueue(MAC, a.fileno(), max_batch=64, flush_usec=300, host_max=16 * 1514) as q:
        def producer(t):
            for _ in range(M):
                assert q.send_async(bytes([2, 0, 0, 0, 0, t]), 0x0800, payload[t]) == 1518
        th = [threading.Thread(target=producer, args=(t,)) for t in range(P)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        q.flush()
        frames, batches, errors = q.stats()
        small_batches, small_frames, gpu_batches = q.paths()
        fb = q.fallbacks()
    rd.join(timeout=60)
    a.close(), b.close()
    assert frames == total and errors == 0 and fb == (0, 0)
    assert na.engine_stats()["host_batches"] == h0
    assert small_batches + gpu_batches == batches and gpu_batches >= 1
    assert small_frames <= 16 * small_batches                  # host batches: at most the minimum
    assert total - small_frames >= 17 * gpu_batches            # GPU batches: above it
    want = Counter(ether_send_frame(oracle, bytes([2, 0, 0, 0, 0, t]), 0x0800, payload[t]) for t in range(P)
                   for _ in range(M))
    assert Counter(got) == want
