"""The C-ABI boundary: the product library loads, exports exactly what include/*.h declare
(nstack_fcs.h: the FCS engine; nstack_txq.h: the batched TX call site; nstack_pcap.h;
nstack_inet.h: the opt-in Internet checksums), and (without a GPU) the batch and device entry
points refuse to compute instead of falling back to the CPU; only the error-less drop-in ether_fcs
answers from its host CRC, counted and reported."""
import ctypes
import os
import re
import subprocess

import pytest

import nstack_amd as na

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "nstack_fcs.h")
HEADERS = [os.path.join(ROOT, "include", h) for h in ("nstack_fcs.h", "nstack_txq.h", "nstack_pcap.h", "nstack_inet.h", "nstack_rxq.h")]


def _declared():
    names = set()
    for h in HEADERS:
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\(", src))
    return sorted(names - {"defined", "void", "__attribute__"})


def test_header_declares_python_exports():
    assert sorted(na.EXPORTS) == _declared()


def test_library_exports_every_declared_symbol():
    lib = na.load()
    out = subprocess.run(["nm", "-D", "--defined-only", na.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (\w+)", out))
    for sym in _declared():
        assert sym in exported, sym
        assert getattr(lib, sym) is not None


def test_dropin_symbol_signature_matches_reference_prototype():
    # src/nstack_ether.h:80: uint32_t ether_fcs(const void *data, size_t bsize);
    src = open(HEADER).read()
    assert re.search(r"uint32_t\s+ether_fcs\s*\(\s*const void \*data,\s*size_t bsize\s*\)\s*;", src)


def test_no_cpu_crc_table_in_product():
    """The product .so embeds no CPU CRC table: the drop-in's host CRC (fcs_host_crc.cpp, its
    last resort only) derives its tables from the polynomial at run time, on first use."""
    data = open(na.LIB_PATH, "rb").read()
    # T0[1] of the reflected table, little-endian; it appears only if a CPU table were embedded.
    assert (0x77073096).to_bytes(4, "little") not in data


def test_code_object_is_gfx950(tmp_path):
    # llvm-objdump --offloading writes the bundles next to its input: give it a copy
    lib = tmp_path / os.path.basename(na.LIB_PATH)
    lib.write_bytes(open(na.LIB_PATH, "rb").read())
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    if out.returncode != 0:
        out = subprocess.run(["strings", na.LIB_PATH], capture_output=True, text=True)
    assert "gfx950" in out.stdout


def _gpu_visible():
    return os.path.exists("/dev/kfd")


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU error path")
def test_fails_loudly_without_gpu():
    lib = na.load()
    rc = lib.ether_fcs_fixed_dev(ctypes.c_void_p(64), 1518, 1518, 1, ctypes.c_void_p(64), None)
    assert rc == -19  # -ENODEV
    with pytest.raises(na.FcsError):
        na.engine_init(0)
    assert lib.ether_fcs_fixed_dev(None, 1518, 1518, 1, None, None) == -22  # -EINVAL first
    # RX verification has no CPU path either
    import numpy as np
    arena = np.zeros(128, dtype=np.uint8)
    off = np.zeros(1, dtype=np.uint64)
    ln = np.full(1, 74, dtype=np.uint32)
    ok = np.zeros(1, dtype=np.uint8)
    assert lib.ether_fcs_verify_host(arena.ctypes.data, 128, off.ctypes.data, ln.ctypes.data, ok.ctypes.data, 1) == -19
    with pytest.raises(na.FcsError):
        na.verify_host(arena, 128, off, ln, ok, 1)


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU error path")
def test_dropin_answers_from_host_crc_without_gpu(golden):
    """the reference ether_fcs (src/ether_fcs.c:4-19) cannot fail, so without a GPU
    the drop-in answers from its host CRC rather than aborting: every golden vector and known answer
    bit-exact, each call counted in fcs_engine_host_fallbacks, the reason on stderr once."""
    code = (
        "import json, sys, nstack_amd as na\n"
        "v = json.loads(sys.stdin.read())\n"
        "arena = open(v['arena_path'], 'rb').read()\n"
        "bad = [i for i, (o, n, c) in enumerate(v['frames']) if na.ether_fcs(arena[o:o + n]) != c]\n"
        "bad += [k for k, c in v['kat'] if na.ether_fcs(bytes.fromhex(k)) != c]\n"
        "print(json.dumps({'bad': bad, 'stats': na.engine_stats()}))\n")
    vec = golden["vectors"]
    frames = [(f["off"], f["len"], f["crc"]) for f in vec["frames"]]
    kat = [(bytes(b"123456789").hex(), 0xCBF43926)]
    payload = {"arena_path": os.path.join(ROOT, "tests", "golden", vec["arena"]), "frames": frames, "kat": kat}
    import json
    p = subprocess.run(["python", "-c", code], input=json.dumps(payload), capture_output=True, text=True,
                       cwd=ROOT, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert res["bad"] == []
    calls = sum(1 for f in frames if f[1] > 0) + len(kat)   # len 0 returns 0 without a GPU call
    assert res["stats"]["host_fallbacks"] == calls
    assert res["stats"]["dropin_retries"] == calls and res["stats"]["dropin_recovered"] == 0
    assert p.stderr.count("answering from the host CRC") == 1


def test_inet_signatures_mirror_reference_functions():
    # src/ip.c:39, src/tcp.c:167-170, src/udp.c:136-139 (argument meaning kept, names prefixed:
    # ip.c stays linked in nstack, so the GPU forms cannot reuse its global symbol)
    src = open(os.path.join(ROOT, "include", "nstack_inet.h")).read()
    assert re.search(r"uint16_t\s+inet_ip_checksum\(const void \*dp, size_t bsize\);", src)
    assert re.search(r"uint16_t\s+inet_tcp_checksum\(uint32_t src, uint32_t dst, const void \*dp, size_t bsize\);", src)
    assert re.search(r"uint16_t\s+inet_udp_checksum\(const void \*dp, size_t len, uint32_t src, uint32_t dst\);", src)


@pytest.mark.skipif(_gpu_visible(), reason="checks the no-GPU error path")
def test_inet_fails_loudly_without_gpu():
    import numpy as np
    lib = na.load()
    arena = np.zeros(64, dtype=np.uint8)
    off = np.zeros(1, dtype=np.uint64)
    ln = np.full(1, 20, dtype=np.uint32)
    out = np.zeros(1, dtype=np.uint16)
    assert lib.inet_csum_batch_host(0, arena.ctypes.data, 64, off.ctypes.data, ln.ctypes.data, None,
                                    out.ctypes.data, 1) == -19
    assert lib.inet_csum_batch_host(7, arena.ctypes.data, 64, off.ctypes.data, ln.ctypes.data, None,
                                    out.ctypes.data, 1) == -22   # unknown mode
    assert lib.inet_csum_batch_host(1, arena.ctypes.data, 64, off.ctypes.data, ln.ctypes.data, None,
                                    out.ctypes.data, 1) == -22   # tcp needs addresses
    assert lib.inet_csum_fixed_dev(0, ctypes.c_void_p(64), 20, 20, 1, None, ctypes.c_void_p(64), None) == -19
    p = subprocess.run(["python", "-c", "import nstack_amd as na; na.ip_checksum(bytes(20))"],
                       capture_output=True, text=True, cwd=ROOT, timeout=120)
    assert p.returncode != 0 and "no usable GPU engine" in p.stderr


@pytest.mark.parametrize("n", [1000, (1 << 20) + 777])   # one thread / the 8-thread split
def test_host_batch_bounds_checked_before_any_work(n):
    """The host-inclusive entry points check every frame against the arena before anything runs
    (nothing written on an error): -EINVAL naming the first bad frame, wherever it sits, for the
    single-threaded check and the 8-thread one (from 1 M frames). Without a GPU, a clean batch
    gets past the check and fails with -ENODEV instead."""
    import numpy as np
    lib = na.load()
    lib.fcs_last_error.restype = ctypes.c_char_p
    ab = 64 * n
    off = np.arange(n, dtype=np.uint64) * 64
    ln = np.full(n, 60, dtype=np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    ok = np.zeros(n, dtype=np.uint8)
    base = ctypes.c_void_p(4096)   # never dereferenced: the check reads only off and len

    def call(kind):
        if kind == "batch":
            return lib.ether_fcs_batch_host(base, ab, off.ctypes.data, ln.ctypes.data, out.ctypes.data, n)
        if kind == "verify":
            return lib.ether_fcs_verify_host(base, ab, off.ctypes.data, ln.ctypes.data, ok.ctypes.data, n)
        return lib.ether_fcs_tx_batch_host(base, ab, off.ctypes.data, ln.ctypes.data, n)

    for kind in ("batch", "verify", "tx"):
        for bad in (0, n // 2, n - 1, (7 * n) // 8 + 1):
            saved = (int(off[bad]), int(ln[bad]))
            for o, L in ((ab + 1, 0), (ab - 10, 11), (2**64 - 8, 16), (64 * bad, 2**32 - 1)):
                off[bad], ln[bad] = o, L
                assert call(kind) == -22, (kind, bad, o, L)
                assert f"frame {bad} " in lib.fcs_last_error().decode()
            off[bad], ln[bad] = saved
        if kind == "tx":   # its FCS must fit too: 61 + 4 > 64 at the arena's end
            ln[n - 1] = 61
            assert call(kind) == -22 and f"frame {n - 1} " in lib.fcs_last_error().decode()
            ln[n - 1] = 60
        if not _gpu_visible():
            assert call(kind) == -19   # clean batch: past the check, no GPU
    assert not out.any() and not ok.any()
