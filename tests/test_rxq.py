"""Batched RX call site (include/nstack_rxq.h) — host logic that needs no GPU.

ether_receive (src/linux/ether.c:180-212): 0 when nothing is queued (:196-198), own-MAC echoes
skipped (:202), host-order ethertype (:206), min(len - 14, bsize) payload bytes copied and len - 14
returned (:208-211). Without a GPU the FCS-trailer mode checks each batch with the library's host
CRC (ether_receive never drops frames for FCS reasons), counted as a fallback.
"""
import os
import socket

import pytest

import nstack_amd as na

OWN = bytes([2, 0, 0, 0, 0, 1])
PEER = bytes([2, 0, 0, 0, 0, 2])


def _gpu_visible():
    return os.path.exists("/dev/kfd")


def frame(src, proto, payload, dst=OWN):
    return dst + src + proto.to_bytes(2, "big") + payload


@pytest.fixture
def pair():
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    b.setblocking(False)
    yield a, b
    a.close(), b.close()


def test_receive_semantics_without_trailer(pair):
    a, b = pair
    with na.RxQueue(b.fileno(), OWN, max_batch=4, trailer=False) as q:
        assert q.receive() == (0, None, None, None, b"")            # nothing queued -> 0
        a.send(frame(PEER, 0x0800, b"A" * 100))
        a.send(frame(OWN, 0x0806, b"echo"))                         # own echo: skipped
        a.send(b"short")                                            # runt: dropped
        a.send(frame(PEER, 0x86DD, b"B" * 1500))                     # 1514 B: the largest kept
        a.send(frame(PEER, 0x0800, b"C" * 1501))                     # 1515 B: oversize, dropped
        a.send(frame(PEER, 0x0806, b"D" * 46))
        n, dst, src, proto, pl = q.receive()
        assert (n, dst, src, proto, pl) == (100, OWN, PEER, 0x0800, b"A" * 100)
        n, _, _, proto, pl = q.receive(bsize=10)                    # len returned, 10 bytes copied
        assert (n, proto, pl) == (1500, 0x86DD, b"B" * 10)
        n, _, _, proto, pl = q.receive()
        assert (n, proto, pl) == (46, 0x0806, b"D" * 46)
        assert q.receive()[0] == 0
        frames, bad, echoes, dropped, batches = q.stats()
        assert (frames, bad, echoes, dropped) == (6, 0, 1, 2) and batches >= 2


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU path")
@pytest.mark.parametrize("host_max", [0, None])
def test_trailer_mode_without_gpu_host_crc_checks(pair, host_max):
    """No GPU: the host CRC checks each batch, so the good frames still come out in order and the
    corrupted one is dropped. host_max 0 (every batch to the GPU): the failed GPU step is answered
    by the host CRC and counted as such; the default GPU minimum: these small batches
    are checked by the host CRC by design, counted apart, with no failure."""
    import struct
    import zlib
    a, b = pair
    good = [frame(PEER, 0x0800 + i, bytes([i]) * (46 + 100 * i)) for i in range(5)]
    with na.RxQueue(b.fileno(), OWN, max_batch=3, trailer=True, host_max=host_max) as q:
        for i, f in enumerate(good):
            t = bytearray(f + struct.pack("<I", zlib.crc32(f)))
            a.send(bytes(t))
            if i == 2:                                               # a corrupted copy
                t[20] ^= 4
                a.send(bytes(t))
        out = []
        while True:
            n, dst, src, proto, pl = q.receive()
            assert n >= 0, n
            if n == 0:
                break
            out.append((proto, pl))
        frames, bad, echoes, dropped, batches = q.stats()
        host_batches, host_frames = q.fallbacks()
        small_batches, small_frames, gpu_batches = q.paths()
    assert out == [(0x0800 + i, bytes([i]) * (46 + 100 * i)) for i in range(5)]
    assert (frames, bad, echoes, dropped) == (6, 1, 0, 0)
    if host_max == 0:
        assert host_batches == batches and host_frames == 6 and small_batches == 0
    else:
        assert (small_batches, small_frames) == (batches, 6) and host_batches == 0 and gpu_batches == 0


def test_bad_arguments():
    lib = na.load()
    assert lib.fcs_rxq_create(-1, OWN, 8, 0) is None
    assert lib.fcs_rxq_create(3, OWN, 0, 0) is None
    assert lib.fcs_rxq_create(3, OWN, 8, 2) is None
    assert lib.fcs_rxq_receive(None, None, None, 0) == -22
