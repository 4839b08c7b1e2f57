"""The TX/RX queues keep ether_send's and ether_receive's contract when the GPU step fails
(SURVEY.md §8b Errors).

ether_send (/root/reference/src/linux/ether.c:214-272) fails only on -EMSGSIZE, a bad handle or
sendto, never because the FCS could not be computed; ether_receive (:180-212) never drops a frame
for FCS reasons. So when a queue's GPU step fails, the batch's FCSs are computed (TX) or checked
(RX) by the library's own host CRC (nstack_amd/csrc/fcs_host_crc.cpp, not the oracle), counted per
queue (fallbacks()) and in fcs_engine_host_batches.

Runs against nstack_amd/libnstack_fcs_faults.so, the test-only -DFCS_FAULT_HOOK build:
fcs_debug_fail_batches(skip, calls) lets the next `skip` queue batch calls (ether_fcs_tx_batch_host,
ether_fcs_verify_host, the mapped-list submit and wait) run and fails the `calls` after them; a
failed wait gives up with its kernel still in flight (the queue then sets the batch's ok array
aside). fcs_debug_late_batches(skip, calls) makes the host batch calls give up after their launch,
with the kernel in flight (the TX queue's arena is reused at once: the engine's kernels never write
into it). Expected frames come from ether_send's layout with the oracle's FCS (TX) and from zlib
(RX); every check is exact."""
import random
import socket
import struct
import threading
import zlib
from collections import Counter

import pytest

import nstack_amd as na

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

MAC = bytes([0x02, 0x42, 0xAC, 0x11, 0x00, 0x02])
OWN = bytes([2, 0, 0, 0, 0, 1])
PEER = bytes([2, 0, 0, 0, 0, 2])


@pytest.fixture(scope="module")
def flib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = na.load_faults()
    yield L
    L.fcs_debug_fail_batches(0, 0)
    L.fcs_debug_late_batches(0, 0)


@pytest.fixture(autouse=True)
def fresh_engine(flib):
    """Each test starts on a fresh engine: failed waits retire resources, and 16 retirements would
    put the host batch forms into host-only mode for the tests after it."""
    flib.fcs_engine_fini()
    yield


def ether_send_frame(oracle, dst, proto, payload, src=MAC):
    frame_size = 14 + max(len(payload), 56) + 4                 # :222-224
    f = dst + src + struct.pack(">H", proto) + payload          # :257-260
    f += b"\0" * (frame_size - 4 - len(f))                      # :261
    return f + struct.pack("<I", oracle.oracle_ether_fcs(f, len(f)))   # :262-263


def run_tx(flib, oracle, max_batch, flush_usec, producers, per, seed, inject=None):
    """producers threads send `per` frames each through one queue of the faults library;
    inject(q) is called once the producers run. Returns (results ok, received == expected,
    stats, fallbacks)."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    plans = []
    for t in range(producers):
        r = random.Random(seed * 100 + t)
        plans.append([(bytes(r.randrange(256) for _ in range(6)), r.choice([0x0800, 0x0806, 0x86DD]),
                       bytes(r.randrange(256) for _ in range(r.choice([0, 1, 55, 56, 57, r.randrange(1501), 1500]))))
                      for _ in range(per)])
    expect = Counter(ether_send_frame(oracle, *x) for p in plans for x in p)
    total = producers * per
    got, results = [], [[] for _ in range(producers)]
    rd = threading.Thread(target=lambda: got.extend(b.recv(2048) for _ in range(total)))
    rd.start()
    # gpu_only: every frame takes a batch's GPU step (the one the faults are injected into)
    with na.TxQueue(MAC, a.fileno(), max_batch=max_batch, flush_usec=flush_usec, lib=flib, gpu_only=True) as q:
        if inject:
            inject(q)

        def producer(t):
            for dst, proto, payload in plans[t]:
                results[t].append((q.send(dst, proto, payload), 14 + max(len(payload), 56) + 4))
        th = [threading.Thread(target=producer, args=(t,)) for t in range(producers)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        q.flush()
        st, fb, why = q.stats(), q.fallbacks(), q.last_error()
    rd.join(timeout=60)
    a.close(), b.close()
    ok_results = all(r == want for rs in results for r, want in rs)
    return ok_results, Counter(got) == expect, st, fb, why


@pytest.mark.parametrize("max_batch,flush_usec,fails", [(1, 0, 3), (64, 200, 2), (1024, 2000, 1)])
def test_tx_gpu_failures_answered_by_host_crc(flib, oracle, max_batch, flush_usec, fails):
    """The first `fails` GPU steps fail: those batches still leave byte-identical to ether_send's
    frames, every sync caller gets frame_size, and exactly `fails` batches are counted."""
    h0 = flib.fcs_engine_host_batches()
    flib.fcs_debug_fail_batches(0, fails)
    ok_res, same, (frames, batches, errors), (hb, hf), why = run_tx(flib, oracle, max_batch, flush_usec, 8, 120,
                                                                   max_batch)
    assert flib.fcs_debug_batch_faults_left() == 0
    assert ok_res and same
    assert frames == 960 and errors == 0
    assert hb == fails and 1 <= hf <= fails * max_batch
    assert flib.fcs_engine_host_batches() - h0 == fails
    assert "injected fault" in why


def test_tx_failure_after_healthy_batches(flib, oracle):
    """Healthy batches first, then a failure in the middle of the stream (its pinned arena is set
    aside and replaced), then healthy again: every frame exact, one batch counted."""
    flib.fcs_debug_fail_batches(5, 1)
    ok_res, same, (frames, batches, errors), (hb, hf), _ = run_tx(flib, oracle, 16, 0, 4, 200, 7)
    assert ok_res and same and errors == 0 and frames == 800
    assert batches > 6 and hb == 1 and 1 <= hf <= 16


@pytest.mark.parametrize("max_batch,producers", [(64, 8), (1024, 8), (4, 1)])
def test_tx_late_failures_with_kernel_in_flight(flib, oracle, max_batch, producers):
    """The GPU step gives up after its launch, the kernel still in flight (a timeout), on the
    first three batches: the engine answers them from the host CRC and retires the stream its
    kernel writes, the queue reuses the arena at once, and every frame that leaves is exact."""
    h0 = flib.fcs_engine_host_batches()
    flib.fcs_debug_late_batches(0, 3)
    ok_res, same, (frames, batches, errors), (hb, hf), why = run_tx(flib, oracle, max_batch, 0, producers, 150, 3)
    assert flib.fcs_debug_batch_faults_left() == 0
    assert ok_res and same and errors == 0 and frames == producers * 150
    assert hb == 3 and flib.fcs_engine_host_batches() - h0 == 3
    assert "injected late fault" in why


def test_retired_kernel_that_stays_busy_does_not_block_the_next_batch(flib, oracle):
    """A small TX batch gives up while its kernel really stays in flight (queued behind a kernel that
    waits for a pinned host word, at most 20 s): the engine answers it from the host CRC and retires
    the small-batch stream. The next small batch runs on a fresh stream without any device-wide
    synchronisation (one there would wait for the held kernel) and is answered by the GPU,
    exact. The held kernel is released 1 s into that call: HIP may give the fresh stream the held
    stream's hardware queue (GPU_MAX_HW_QUEUES = 4), and then the batch waits for the release; either
    way it returns well inside the engine's 10 s timeout."""
    import ctypes
    import threading
    import time
    word = flib.fcs_host_alloc(64)
    arena = flib.fcs_host_alloc(8 * 1536)
    assert word and arena
    ctypes.memset(word, 0, 64)
    n, stride = 4, 1536
    off = (ctypes.c_uint64 * n)(*[i * stride for i in range(n)])
    ln = (ctypes.c_uint32 * n)(*[60 + 300 * i for i in range(n)])
    rng = random.Random(5)
    flib.fcs_last_error.restype = ctypes.c_char_p

    def fill_and_expect():
        body = [bytes(rng.randrange(256) for _ in range(ln[i])) for i in range(n)]
        for i in range(n):
            ctypes.memmove(arena + off[i], body[i], ln[i])
        return [struct.pack("<I", oracle.oracle_ether_fcs(b, len(b))) for b in body]

    def got():
        return [ctypes.string_at(arena + off[i] + ln[i], 4) for i in range(n)]

    release = threading.Timer(1.0, lambda: ctypes.memset(word, 0xFF, 4))
    try:
        want = fill_and_expect()
        h0 = flib.fcs_engine_host_batches()
        flib.fcs_debug_hold_small(word)          # the next small launch waits behind the hold kernel
        flib.fcs_debug_late_batches(0, 1)        # ... and its call gives up with it in flight
        assert flib.ether_fcs_tx_batch_host(arena, 8 * 1536, off, ln, n) == 0
        assert flib.fcs_engine_host_batches() - h0 == 1 and got() == want   # host CRC answer
        want = fill_and_expect()
        s0 = flib.fcs_debug_device_syncs()
        release.start()
        t0 = time.monotonic()
        assert flib.ether_fcs_tx_batch_host(arena, 8 * 1536, off, ln, n) == 0
        dt = time.monotonic() - t0
        assert flib.fcs_engine_host_batches() - h0 == 1, flib.fcs_last_error()   # the GPU answered
        assert got() == want
        assert flib.fcs_debug_device_syncs() == s0           # nothing waited on the retired stream
        assert dt < 5.0, dt
    finally:
        release.cancel()
        ctypes.memset(word, 0xFF, 4)             # release the held kernel (if the timer has not)
        flib.fcs_engine_fini()                   # waits for it (released) before freeing
        flib.fcs_host_free(arena)
        flib.fcs_host_free(word)


def rx_frame(payload, proto=0x0800):
    body = OWN + PEER + proto.to_bytes(2, "big") + payload + bytes(max(0, 56 - len(payload)))
    return body + struct.pack("<I", zlib.crc32(body))


def rx_stream(n, seed):
    rng = random.Random(seed)
    sent, good = [], []
    for i in range(n):
        pl = i.to_bytes(4, "little") + bytes(rng.randrange(256) for _ in range(rng.choice([0, 40, 700, 1400])))
        f = bytearray(rx_frame(pl, 0x0800 + (i & 7)))
        if rng.random() < 0.1:
            f[rng.randrange(len(f))] ^= 1 << rng.randrange(8)      # corrupted anywhere, trailer included
        else:
            good.append((0x0800 + (i & 7), pl + bytes(max(0, 56 - len(pl)))))
        sent.append(bytes(f))
    return sent, good


def drain(q):
    out = []
    while True:
        n, dst, src, proto, pl = q.receive()
        assert n >= 0, n                                # never a GPU error code
        if n == 0:
            return out
        assert dst == OWN and src == PEER
        out.append((proto, pl))


@pytest.mark.parametrize("skip,fails", [(0, 1), (0, 2), (1, 1), (0, 3), (2, 4)])
def test_rx_gpu_failures_checked_by_host_crc(flib, skip, fails):
    """Submit failures (nothing launched) and wait failures (kernel left in flight, ok array set
    aside) at the start of the stream: the good frames come out in order, every corrupted one is
    dropped, and the host-checked batches are counted."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    b.setblocking(False)
    sent, good = rx_stream(400, 31 * skip + fails)
    for f in sent:
        a.send(f)
    h0 = flib.fcs_engine_host_batches()
    flib.fcs_debug_fail_batches(skip, fails)
    with na.RxQueue(b.fileno(), OWN, max_batch=16, trailer=True, lib=flib, host_max=0) as q:
        got = drain(q)
        frames, bad, echoes, dropped, batches = q.stats()
        hb, hf = q.fallbacks()
    flib.fcs_debug_fail_batches(0, 0)
    a.close(), b.close()
    assert got == good
    assert frames == len(sent) and bad == len(sent) - len(good) and dropped == 0
    assert 1 <= hb <= fails and hb <= batches and hf <= 16 * hb
    assert flib.fcs_engine_host_batches() - h0 == hb


def test_rx_wait_failure_then_gpu_again(flib):
    """One batch's wait fails with its kernel in flight; later batches go back to the GPU (into
    the fresh ok array) and are not counted."""
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 4 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 4 << 20)
    b.setblocking(False)
    sent, good = rx_stream(10, 5)
    for f in sent:                      # one batch: submit (call 1) runs, its wait (call 2) fails
        a.send(f)
    flib.fcs_debug_fail_batches(1, 1)
    with na.RxQueue(b.fileno(), OWN, max_batch=16, trailer=True, lib=flib, host_max=0) as q:
        got = drain(q)
        assert flib.fcs_debug_batch_faults_left() == 0
        assert q.fallbacks() == (1, 10)
        sent2, good2 = rx_stream(300, 6)
        for f in sent2:
            a.send(f)
        got2 = drain(q)
        assert q.fallbacks() == (1, 10)   # the GPU checked everything after the failure
    a.close(), b.close()
    assert got == good and got2 == good2


def test_rx_live_sender_with_failures(flib):
    """A sender thread pushes bursts while the consumer arms a batch failure every few frames: the
    good frames come out once, in order, whatever mix of GPU and host checks served them."""
    import time
    a, b = socket.socketpair(socket.AF_UNIX, socket.SOCK_DGRAM)
    a.setsockopt(socket.SOL_SOCKET, socket.SO_SNDBUF, 8 << 20)
    b.setsockopt(socket.SOL_SOCKET, socket.SO_RCVBUF, 8 << 20)
    b.setblocking(False)
    sent, good = rx_stream(2000, 77)

    def sender():
        for k in range(0, len(sent), 97):
            for f in sent[k:k + 97]:
                a.send(f)
            time.sleep(0.0005 * (k % 3))

    th = threading.Thread(target=sender)
    th.start()
    got = []
    deadline = time.time() + 60
    with na.RxQueue(b.fileno(), OWN, max_batch=32, trailer=True, lib=flib, host_max=0) as q:
        i = 0
        while len(got) < len(good) and time.time() < deadline:
            if i % 50 == 0:
                flib.fcs_debug_fail_batches(i % 3, 1)
            i += 1
            n, dst, src, proto, pl = q.receive()
            assert n >= 0, n
            if n:
                got.append((proto, pl))
        th.join()
        got += drain(q)
        hb, _ = q.fallbacks()
    flib.fcs_debug_fail_batches(0, 0)
    a.close(), b.close()
    assert got == good
    assert hb >= 1
