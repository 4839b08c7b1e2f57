"""The TX queue's AF_PACKET sink (fcs_txq_sink_packet, include/nstack_txq.h) against ether_send's
addressing and result contract, without CAP_NET_RAW or a GPU.

ether_send (/root/reference/src/linux/ether.c:244-255) sends each frame with sendto to a
sockaddr_ll { AF_PACKET, htons(proto), the interface's ifindex, halen 6, sll_addr = dst }, every
other field zero, length sizeof(struct sockaddr_ll); a failed sendto makes that frame's result
-errno (:265-269), else it is the bytes sent. The sink does the same for a whole batch with
sendmmsg, and sends a batch of one frame (a synchronous sender's own frame) with sendto, exactly
ether_send's call: tests/c/packet_sink_check defines sendmmsg and sendto itself (the executable's definition comes first
in the dynamic linker's lookup scope, so the library binds to it), records every message and answers
from a script of partial sends, errors and EINTR. Expected values are built here from ether.c's
layout, field by field."""
import json
import os
import shutil
import socket
import struct
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c")
BIN = os.path.join(CDIR, "packet_sink_check")
PROTOS = (0x0800, 0x0806, 0x86DD, 0x88CC)


@pytest.fixture(scope="module")
def check():
    if shutil.which("gcc") and os.path.exists(os.path.join(ROOT, "nstack_amd", "libnstack_fcs.so")):
        subprocess.run(["make", "-s", "-C", CDIR], check=True, capture_output=True)
    if not os.path.exists(BIN):
        pytest.skip("tests/c/packet_sink_check not built")
    return BIN


def frame_of(i):
    """Frame i as packet_sink_check builds it (ether_send's layout): dst, proto, frame_size."""
    bsize = (i * 397) % 1501
    dst = bytes([(0x02 | (i & 0xF0)) & 255, i & 255, (i >> 8) & 255, 0xA5, (i * 7) & 255, (255 - i) & 255])
    return dst, PROTOS[i & 3], 14 + max(bsize, 56) + 4


def sockaddr_ll(dst, proto, ifindex):
    """struct sockaddr_ll as ether.c:244-255 initialises it (designated initialiser: the rest zero)."""
    return (struct.pack("<H", socket.AF_PACKET) + struct.pack(">H", proto) + struct.pack("<i", ifindex)
            + struct.pack("<HBB", 0, 0, 6) + dst + b"\0\0")


def run(check, n, ifindex, script):
    out = subprocess.run([check, str(n), str(ifindex), script], capture_output=True, text=True, timeout=60,
                         check=True).stdout
    recs = [json.loads(x) for x in out.splitlines()]
    return ([r for r in recs if "call" in r], [r for r in recs if "msg" in r], [r for r in recs if "res" in r][0])


@pytest.mark.parametrize("n,ifindex", [(1, 2), (7, 9), (64, 3), (500, 123456)])
def test_every_frame_addressed_as_ether_send(check, n, ifindex):
    calls, msgs, res = run(check, n, ifindex, "A")
    assert len(calls) == 1 and calls[0]["fd"] == 77 and calls[0]["flags"] == 0 and calls[0]["vlen"] == n
    assert [m["msg"] for m in msgs] == list(range(n))
    for i, m in enumerate(msgs):
        dst, proto, size = frame_of(i)
        assert m["namelen"] == 20                                           # sizeof(struct sockaddr_ll)
        assert bytes.fromhex(m["name"]) == sockaddr_ll(dst, proto, ifindex), i
        assert m["iovlen"] == 1 and m["len"] == size and m["control"] == 0
        assert bytes.fromhex(m["head"]) == dst + bytes([2, 0x42, 0xAC, 0x11, 0, 2]) + struct.pack(">H", proto)
    assert res["res"] == res["sizes"] == [frame_of(i)[2] for i in range(n)]


@pytest.mark.parametrize("script,expect", [
    # accept 2, then the 3rd fails with ENOBUFS, then EINTR is retried, then 1, then the rest
    ("2,E105,I,1,A", ["ok", "ok", -105, "ok", "ok", "ok", "ok", "ok"]),
    # every message fails on its own: each frame gets its -errno, the queue goes on
    ("E1,E11,E90,E105,E100,E101,E113,E22", [-1, -11, -90, -105, -100, -101, -113, -22]),
    # zero accepted is not an error: the same frames are offered again
    ("0,0,3,E32,A", ["ok", "ok", "ok", -32, "ok", "ok", "ok", "ok"]),
    ("I,I,I,A", ["ok"] * 8),
])
def test_partial_sends_and_errors_map_per_frame(check, script, expect):
    """sendto's per-frame contract (:265-269) through sendmmsg's partial returns: frames the kernel
    accepted report their length, a failing frame -errno, and the frames after it are still sent."""
    n = len(expect)
    calls, msgs, res = run(check, n, 5, script)
    sizes = [frame_of(i)[2] for i in range(n)]
    assert res["res"] == [sizes[i] if e == "ok" else e for i, e in enumerate(expect)]
    sent_idx = [i for i, e in enumerate(expect) if e == "ok"]
    assert len(msgs) == len(sent_idx)
    for m, i in zip(msgs, sent_idx):
        dst, proto, size = frame_of(i)
        assert bytes.fromhex(m["name"]) == sockaddr_ll(dst, proto, 5) and m["len"] == size
    # every call offers exactly the frames not yet answered, in order
    left = n
    for c in calls:
        assert c["vlen"] == left
        e = c["entry"]
        if e.startswith("E"):
            left -= 1
        elif e == "I":
            pass
        elif e == "A":
            left = 0
        else:
            left -= min(int(e), left)
    assert left == 0


@pytest.mark.parametrize("script,expect", [("A", "ok"), ("E105", -105), ("I,A", "ok"), ("I,I,E90", -90)])
def test_single_frame_is_one_sendto(check, script, expect):
    """A batch of one (fcs_txq_send's own frame): one sendto with ether_send's sockaddr_ll, EINTR
    retried, any other error the frame's -errno."""
    calls, msgs, res = run(check, 1, 7, script)
    assert all(c.get("kind") == "sendto" and c["fd"] == 77 and c["flags"] == 0 for c in calls)
    dst, proto, size = frame_of(0)
    assert res["res"] == [size if expect == "ok" else expect]
    assert len(msgs) == (1 if expect == "ok" else 0)
    for m in msgs:
        assert m["namelen"] == 20 and bytes.fromhex(m["name"]) == sockaddr_ll(dst, proto, 7) and m["len"] == size
