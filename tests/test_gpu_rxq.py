"""Batched RX call site with GPU FCS verification (include/nstack_rxq.h).

Frames are built as ether_send builds them (src/linux/ether.c:257-263: header, payload, zero pad,
little-endian FCS over the rest) so the trailer is exactly what a link with rx-fcs delivers; a few
are corrupted. Expected: the good frames come out in order with the trailer stripped, the
corrupted ones are counted and never handed out."""
import random
import socket
import struct
import zlib

import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu

OWN = bytes([2, 0, 0, 0, 0, 1])
PEER = bytes([2, 0, 0, 0, 0, 2])


def ether_send_frame(payload, proto=0x0800, src=PEER, dst=OWN):
    body = dst + src + proto.to_bytes(2, "big") + payload + bytes(max(0, 56 - len(payload)))
    return body + struct.pack("<I", zlib.crc32(body))


@pytest.mark.parametrize("host_max", [0, None])   # every batch on the GPU / the default GPU minimum
@pytest.mark.parametrize("max_batch", [1, 7, 64])
def test_rx_verify_drops_corrupted_frames(max_batch, host_max):
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    b.setblocking(False)
    rng = random.Random(max_batch)
    sent, good = [], []
    for i in range(300):
        pl = bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 46, 100, 576, 1480, 1500])))
        f = bytearray(ether_send_frame(pl, proto=0x0800 + (i & 7)))
        kind = rng.random()
        if kind < 0.1:
            f[rng.randrange(len(f))] ^= 1 << rng.randrange(8)      # corrupted anywhere, trailer included
        elif kind < 0.15:
            f[6:12] = OWN                                           # own echo (refresh its FCS)
            f[-4:] = struct.pack("<I", zlib.crc32(bytes(f[:-4])))
        else:
            good.append((max(len(pl), 56), 0x0800 + (i & 7), pl + bytes(max(0, 56 - len(pl)))))
        sent.append(bytes(f))
    for f in sent:
        a.send(f)
    got = []
    with na.RxQueue(b.fileno(), OWN, max_batch=max_batch, trailer=True, host_max=host_max) as q:
        while True:
            n, dst, src, proto, pl = q.receive()
            if n == 0:
                break
            assert n > 0, n
            assert dst == OWN and src == PEER
            got.append((n, proto, pl))
        frames, bad, echoes, dropped, batches = q.stats()
        small_batches, small_frames, gpu_batches = q.paths()
        assert q.fallbacks() == (0, 0)                          # no GPU check failed
        assert small_batches + gpu_batches == batches
        if host_max == 0:
            assert gpu_batches == batches                       # the GPU checked every batch
    a.close(), b.close()
    assert got == good
    assert frames == len(sent) and dropped == 0
    assert bad + echoes + len(good) == len(sent) and bad > 0 and echoes > 0


@pytest.mark.parametrize("host_max", [0, None])   # every batch on the GPU / the default GPU minimum
@pytest.mark.parametrize("max_batch", [16, 64])
def test_rx_pipeline_with_live_sender(max_batch, host_max):
    """Frames arriving while batches are checked: the queue overlaps the GPU check of one batch
    with the recvmmsg of the next (two buffers). A sender thread pushes bursts with pauses, so
    the receiver meets full, partial and empty queues; every good frame must come out once, in
    order, and no corrupted one."""
    import threading
    import time
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    b.setblocking(False)
    rng = random.Random(1000 + max_batch)
    frames, good = [], []
    for i in range(3000):
        pl = i.to_bytes(4, "little") + bytes(rng.randrange(256) for _ in range(rng.choice([0, 60, 700, 1400])))
        f = bytearray(ether_send_frame(pl))
        if rng.random() < 0.05:
            f[rng.randrange(len(f))] ^= 0x10
        else:
            good.append(pl + bytes(max(0, 56 - len(pl))))
        frames.append(bytes(f))

    def sender():
        for k in range(0, len(frames), 97):
            for f in frames[k:k + 97]:
                a.send(f)
            time.sleep(0.0005 * (k % 3))

    th = threading.Thread(target=sender)
    th.start()
    got = []
    deadline = time.time() + 60
    with na.RxQueue(b.fileno(), OWN, max_batch=max_batch, trailer=True, host_max=host_max) as q:
        while len(got) < len(good) and time.time() < deadline:
            n, dst, src, proto, pl = q.receive()
            assert n >= 0, n
            if n:
                got.append(pl)
        th.join()
        while True:   # the corrupted frames after the last good one
            n, *_ = q.receive()
            assert n >= 0, n
            if n == 0:
                break
            got.append(None)
        st = q.stats()
        assert q.fallbacks() == (0, 0)
    a.close(), b.close()
    assert got == good
    assert st[1] == len(frames) - len(good)


def test_rx_destroy_with_batches_in_flight():
    """Closing the queue while a batch's check is still on the GPU (the pipeline launches the
    next batch before handing out the current one) waits for it and frees cleanly; a new queue
    on the same socket then receives the rest."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    b.setblocking(False)
    for i in range(200):
        a.send(ether_send_frame(i.to_bytes(4, "little") * 20))
    with na.RxQueue(b.fileno(), OWN, max_batch=16, trailer=True, host_max=0) as q:
        n, *_rest, pl = q.receive()
        assert n > 0 and pl[:4] == (0).to_bytes(4, "little")
    got = 0
    with na.RxQueue(b.fileno(), OWN, max_batch=64, trailer=True, host_max=0) as q:
        while q.receive()[0] > 0:
            got += 1
    a.close(), b.close()
    assert 0 < got <= 199 - 15   # the first queue took at least its first two batches
