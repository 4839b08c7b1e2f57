"""The ether_send call-site change is an artifact, not prose.

integration/ether_txq.patch is the edit INTEGRATION.md §2 describes, as a unified diff against the
reference's src/linux/ether.c (/root/reference/src/linux/ether.c:214-272 for ether_send, :106-178
for ether_init / ether_deinit): one fcs_txq_t per ether handle, created next to the AF_PACKET
socket, and ether_send's body after the -EMSGSIZE and handle checks reduced to fcs_txq_send().

CPU only, and only where the reference tree is present (this container; never the GPU box). The
reference is never modified: its src/, include/ and config.h are copied to a temporary directory,
where the patch must apply cleanly (patch --dry-run, git apply --check) and the patched file must
compile with the reference Makefile's flags (Makefile:4-6) against the reference headers and
include/nstack_txq.h (gcc -fsyntax-only).
"""
import os
import shutil
import subprocess
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
PATCH = os.path.join(ROOT, "integration", "ether_txq.patch")

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(REF, "src", "linux", "ether.c")),
                                reason="reference tree not present (GPU box)")


@pytest.fixture()
def tree():
    d = tempfile.mkdtemp(prefix="nstack_patch_")
    try:
        for x in ("src", "include"):
            shutil.copytree(os.path.join(REF, x), os.path.join(d, x))
        shutil.copy(os.path.join(REF, "config.h"), d)
        yield d
    finally:
        shutil.rmtree(d, ignore_errors=True)


def _run(cmd, cwd):
    return subprocess.run(cmd, cwd=cwd, capture_output=True, text=True)


def test_patch_touches_only_the_call_site_file():
    with open(PATCH) as f:
        heads = [l for l in f if l.startswith(("--- ", "+++ "))]
    assert heads == ["--- a/src/linux/ether.c\n", "+++ b/src/linux/ether.c\n"]


def test_patch_applies_cleanly(tree):
    r = _run(["patch", "-p1", "--dry-run", "-i", PATCH], tree)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "fuzz" not in r.stdout.lower() and "offset" not in r.stdout.lower()
    assert _run(["git", "init", "-q", "."], tree).returncode == 0
    r = _run(["git", "apply", "--check", PATCH], tree)
    assert r.returncode == 0, r.stderr


def test_patched_call_site_compiles_against_the_reference_headers(tree):
    assert _run(["patch", "-p1", "-s", "-i", PATCH], tree).returncode == 0
    with open(os.path.join(tree, "src", "linux", "ether.c")) as f:
        src = f.read()
    assert src.count("fcs_txq_send(eth->el_txq, dst, proto, buf, bsize)") == 1
    assert "ether_fcs(" not in src.split("int ether_send(")[1]      # no per-frame FCS left at the call site
    assert "fcs_txq_create(" in src and "fcs_txq_destroy(eth->el_txq)" in src
    r = _run(["gcc", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "--std=gnu99",
              "-pthread", "-include", "config.h", "-I", "include", "-I", os.path.join(ROOT, "include"),
              "src/linux/ether.c"], tree)
    assert r.returncode == 0, r.stderr
