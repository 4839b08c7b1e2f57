"""ThreadSanitizer and AddressSanitizer + UBSan runs of the TX and RX queues' host code
(tools/tsan/run.sh; CPU only).

The multi-producer reservation, hand-offs and flusher of fcs_txq.cpp are built with
-fsanitize=thread (and, separately, -fsanitize=address,undefined) against a stubbed GPU step
(tools/tsan/gpu_stub.cpp) and driven by 1 to 4096 producers' worth of frames at several queue
capacities and linger times; the run fails on any sanitizer report (leaks included under ASan) or
a lost or duplicated frame. The RX queue (fcs_rxq.cpp) receives good, corrupted, runt, oversize
and own-MAC frames over an AF_UNIX socketpair with the stubbed check failing every third call or
never, and with another thread changing its GPU minimum; every good frame must come out once, in
order, with exact drop counters. Under ASan the pcap reader (fcs_pcap.cpp) also takes 3000
corrupted captures (bit flips, bad record lengths, truncation, the other byte order, pcapng):
every call returns a count or -errno without touching memory outside its buffers. Keeping it in the CPU suite also keeps the engine's host-only headers
buildable without ROCm (the harness compiles them with plain g++).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_txq_tsan_clean(tmp_path, san):
    env = dict(os.environ, TMPDIR=str(tmp_path), SAN=san)
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "tsan", "run.sh")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert f"{san}: clean" in r.stdout
