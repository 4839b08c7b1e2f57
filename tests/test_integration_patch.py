"""The call-site changes are artifacts, not prose.

integration/ether_txq.patch is the ether_send edit INTEGRATION.md §2 describes, as a unified diff
against the reference's src/linux/ether.c (/root/reference/src/linux/ether.c:214-272 for ether_send,
:106-178 for ether_init / ether_deinit): one fcs_txq_t per ether handle, created next to the
AF_PACKET socket, and ether_send's body after the -EMSGSIZE and handle checks reduced to
fcs_txq_send(). integration/ether_rxq.patch is the ether_receive edit (:180-212): one fcs_rxq_t per
handle, created in ether_init after the socket is bound, destroyed in ether_deinit and on ether_init's
failure path, and ether_receive's body after the handle check reduced to fcs_rxq_receive() with the
reference's return convention (-1 and errno on a socket error). The two patches touch separate lines,
so either applies with or without the other, in either order.

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
RX_PATCH = os.path.join(ROOT, "integration", "ether_rxq.patch")
CFLAGS = ["-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter", "--std=gnu99", "-pthread",
          "-include", "config.h", "-I", "include", "-I", os.path.join(ROOT, "include")]

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


@pytest.mark.parametrize("patch", [PATCH, RX_PATCH])
def test_patch_touches_only_the_call_site_file(patch):
    with open(patch) as f:
        heads = [l for l in f if l.startswith(("--- ", "+++ "))]
    assert heads == ["--- a/src/linux/ether.c\n", "+++ b/src/linux/ether.c\n"]


@pytest.mark.parametrize("patch", [PATCH, RX_PATCH])
def test_patch_applies_cleanly(tree, patch):
    r = _run(["patch", "-p1", "--dry-run", "-i", patch], tree)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "FAILED" not in r.stdout and "fuzz" not in r.stdout.lower() and "offset" not in r.stdout.lower()
    assert _run(["git", "init", "-q", "."], tree).returncode == 0
    r = _run(["git", "apply", "--check", patch], tree)
    assert r.returncode == 0, r.stderr


def test_patched_call_site_compiles_against_the_reference_headers(tree):
    assert _run(["patch", "-p1", "-s", "-i", PATCH], tree).returncode == 0
    with open(os.path.join(tree, "src", "linux", "ether.c")) as f:
        src = f.read()
    assert src.count("fcs_txq_send(eth->el_txq, dst, proto, buf, bsize)") == 1
    assert "ether_fcs(" not in src.split("int ether_send(")[1]      # no per-frame FCS left at the call site
    assert "fcs_txq_create(" in src and "fcs_txq_destroy(eth->el_txq)" in src
    r = _run(["gcc"] + CFLAGS + ["src/linux/ether.c"], tree)
    assert r.returncode == 0, r.stderr


def test_patched_rx_call_site_compiles_against_the_reference_headers(tree):
    assert _run(["patch", "-p1", "-s", "-i", RX_PATCH], tree).returncode == 0
    with open(os.path.join(tree, "src", "linux", "ether.c")) as f:
        src = f.read()
    body = src.split("int ether_receive(")[1].split("int ether_send(")[0]
    assert body.count("fcs_rxq_receive(ether_rxq[handle]") == 1
    assert "recvfrom(" not in body                                  # no per-frame receive left
    assert "errno = -retval;" in body and "return -1;" in body     # the reference's error convention
    assert "fcs_rxq_create(eth->el_fd, eth->el_mac" in src and src.count("fcs_rxq_destroy(ether_rxq[handle])") == 2
    r = _run(["gcc"] + CFLAGS + ["src/linux/ether.c"], tree)
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("order", [(PATCH, RX_PATCH), (RX_PATCH, PATCH)])
def test_both_patches_apply_in_either_order_and_compile(tree, order):
    """The TX and RX edits touch separate lines of src/linux/ether.c: whichever is applied first, the
    second applies without fuzz (line offsets only), and the file with both compiles."""
    assert _run(["git", "init", "-q", "."], tree).returncode == 0
    for p in order:
        r = _run(["patch", "-p1", "-i", p], tree)
        assert r.returncode == 0 and "fuzz" not in r.stdout.lower() and "FAILED" not in r.stdout, r.stdout + r.stderr
    with open(os.path.join(tree, "src", "linux", "ether.c")) as f:
        src = f.read()
    assert "fcs_txq_send(eth->el_txq" in src and "fcs_rxq_receive(ether_rxq[handle]" in src
    r = _run(["gcc"] + CFLAGS + ["src/linux/ether.c"], tree)
    assert r.returncode == 0, r.stderr
