"""The library's host code under AddressSanitizer + UBSan on the GPU (tools/asan): a C driver runs
every host-facing entry point (drop-in, host batch forms in pageable and pinned memory, TX in place,
RX verify, argument errors, the TX and RX queues, the Internet-checksum host batch) against a build
whose host side is instrumented, then, against the fault-hook build, the recovery paths (failed
and timed-out drop-in attempts, host batches that give up with the kernel in flight, a small batch
held behind a busy kernel, RX checks failing after their launch). Any sanitizer report or wrong
result fails. Built by __graft_entry__.build() (make -C tools/asan)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tools", "asan")


@pytest.mark.gpu
def test_host_code_clean_under_asan_and_ubsan():
    for exe in ("driver", "driver_faults"):
        if not os.path.exists(os.path.join(ASAN, exe)):
            pytest.fail(f"tools/asan/{exe} not built (make -C tools/asan)")
    r = subprocess.run(["bash", os.path.join(ASAN, "run.sh")], capture_output=True, text=True, timeout=660)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("asan driver: ok (0 failures)") == 2, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error:" not in out, out[-4000:]
