"""The link-level drop-in (/root/reference/Makefile:13,42-43).

tests/c/dropin_caller.c declares `uint32_t ether_fcs(const void *data, size_t bsize);` verbatim as
src/nstack_ether.h:80 does, includes no engine header, and is linked with -lnstack_fcs where the
reference links ether_fcs.o. CPU tests: the caller leaves ether_fcs undefined, the dynamic linker
binds it to libnstack_fcs.so, and nothing else could define it (the same link without -lnstack_fcs
fails). GPU test: the linked binary's FCS of every golden vector equals the reference's.
"""
import json
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CDIR = os.path.join(ROOT, "tests", "c")
BIN = os.path.join(CDIR, "dropin_caller")
GOLDEN = os.path.join(ROOT, "tests", "golden")


@pytest.fixture(scope="module")
def caller():
    if shutil.which("gcc") and os.path.exists(os.path.join(ROOT, "nstack_amd", "libnstack_fcs.so")):
        subprocess.run(["make", "-s", "-C", CDIR], check=True, capture_output=True)
    if not os.path.exists(BIN):
        pytest.skip("tests/c/dropin_caller not built (build() makes it)")
    return BIN


def test_caller_leaves_ether_fcs_to_the_library(caller):
    out = subprocess.run(["nm", "-D", caller], capture_output=True, text=True, check=True).stdout
    assert any(l.split()[-2:] == ["U", "ether_fcs"] for l in out.splitlines()), out
    ldd = subprocess.run(["ldd", caller], capture_output=True, text=True, check=True).stdout
    assert "libnstack_fcs.so" in ldd and "not found" not in ldd.split("libnstack_fcs.so", 1)[1].splitlines()[0]


def test_dynamic_linker_binds_ether_fcs_to_libnstack_fcs(caller):
    env = dict(os.environ, LD_BIND_NOW="1", LD_DEBUG="bindings")
    p = subprocess.run([caller, os.path.join(GOLDEN, "vectors.bin")], input="", capture_output=True,
                       text=True, env=env, timeout=60)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [l for l in p.stderr.splitlines() if "`ether_fcs'" in l]
    assert lines and all("libnstack_fcs.so" in l.split(" to ", 1)[1] for l in lines), lines


def test_no_other_definition_of_ether_fcs(tmp_path):
    if not shutil.which("gcc"):
        pytest.skip("no gcc")
    p = subprocess.run(["gcc", "-o", str(tmp_path / "x"), os.path.join(CDIR, "dropin_caller.c")],
                       capture_output=True, text=True)
    assert p.returncode != 0 and "ether_fcs" in p.stderr


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU path")
def test_linked_caller_without_gpu_gets_host_crc_answers(caller):
    """Without a GPU the linked caller still gets ether_fcs's answers (the reference
    cannot fail): the drop-in's host CRC, reported once on stderr, never an abort."""
    vec = json.load(open(os.path.join(GOLDEN, "vectors.json")))
    frames = vec["frames"][:40]
    inp = "".join(f"{f['off']} {f['len']}\n" for f in frames)
    p = subprocess.run([caller, os.path.join(GOLDEN, vec["arena"])], input=inp, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    assert [int(x, 16) for x in p.stdout.split()] == [f["crc"] for f in frames]
    assert p.stderr.count("answering from the host CRC") == 1


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists("/dev/kfd"), reason="needs the GPU box")
def test_linked_caller_golden_vectors(caller):
    vec = json.load(open(os.path.join(GOLDEN, "vectors.json")))
    frames = vec["frames"]
    inp = "".join(f"{f['off']} {f['len']}\n" for f in frames)
    p = subprocess.run([caller, os.path.join(GOLDEN, vec["arena"])], input=inp, capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    got = [int(x, 16) for x in p.stdout.split()]
    assert got == [f["crc"] for f in frames]
    kat = json.load(open(os.path.join(GOLDEN, "kat.json")))
    nine = next(c for c in kat["cases"] if c.get("hex") == b"123456789".hex())
    assert nine["crc"] == 0xCBF43926
