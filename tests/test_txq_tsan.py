"""ThreadSanitizer run of the TX queue's host code (tools/tsan/run.sh; CPU only).

The multi-producer reservation, hand-offs and flusher of fcs_txq.cpp are built with
-fsanitize=thread against a stubbed GPU step (tools/tsan/gpu_stub.cpp) and driven by 1 to 4096
producers' worth of frames at several queue capacities and linger times; the run fails on any TSan
report or a lost or duplicated frame. Keeping it in the CPU suite also keeps the engine's
host-only headers buildable without ROCm (the harness compiles them with plain g++).
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_txq_tsan_clean(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "tsan", "run.sh")], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "tsan: clean" in r.stdout
