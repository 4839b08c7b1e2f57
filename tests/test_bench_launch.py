"""bench.py --gpus N is authoritative (BASELINE configs[4]).

Without a launcher (no WORLD_SIZE), `bench.py --gpus N` starts the N ranks itself under
torch.distributed.run from a parent that has made no GPU call; under a launcher whose world size
differs from N it exits 1. Every rank's device identity is gathered into config.devices, ranks sharing
a GPU labelled as such. CPU only: --dry-run stops after the rendezvous (gloo), before any GPU call."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def _env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(extra)
    return env


def _json_line(out: str):
    lines = [x for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.timeout(180)
@pytest.mark.parametrize("n", [2, 3])
def test_gpus_n_self_launches_n_ranks(n):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       env=_env(), capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == n and rec["dry_run"] is True
    devs = rec["config"]["devices"]
    assert [d["rank"] for d in devs] == list(range(n))
    assert [d["local_rank"] for d in devs] == list(range(n))
    assert rec["config"]["distinct_devices"] == n


@pytest.mark.timeout(60)
def test_world_size_mismatch_exits_1():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"), capture_output=True, text=True, timeout=50)
    assert r.returncode == 1
    assert "WORLD_SIZE=2 but --gpus 4" in r.stderr
    assert not [x for x in r.stdout.splitlines() if x.startswith("{")]


@pytest.mark.timeout(60)
def test_single_gpu_default_needs_no_launcher():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--dry-run"], env=_env(),
                       capture_output=True, text=True, timeout=50)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = _json_line(r.stdout)
    assert rec["n_gpus"] == 1 and len(rec["config"]["devices"]) == 1


def test_label_devices_marks_shared_gpus():
    e = [{"rank": 0, "pci": "0000:05:00"}, {"rank": 1, "pci": "0000:05:00"}, {"rank": 2, "pci": "0000:15:00"}]
    devs, distinct = bench.label_devices(e)
    assert distinct == 2
    assert [d["shares_gpu_with_ranks"] for d in devs] == [[1], [0], []]
