"""Every measurement-only switch documented in DESIGN.md §4.6 still compiles for gfx950.

The switches select ablations and A/B variants of the live kernels (tools/variants.sh builds them
into tools/variants/ for tools/ab.py); nothing in `make` or the product sets them. Compiling each
set here keeps them from rotting as the live kernels change. CPU only: hipcc cross-compiles.
"""
import os
import shutil
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "nstack_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"

# (translation unit, flag set): switches that combine are built together to keep this quick.
VARIANTS = [
    ("fcs_kernel.hip", "-DFCS_NT"),
    ("fcs_kernel.hip", "-DFCS_ABL_NOLDS -DFCS_ABL_NOALIGN -DFCS_ABL_NOFINAL"),
    ("fcs_kernel.hip", "-DFCS_ABL_NOCOMPUTE"),
    ("fcs_kernel.hip", "-DFCS_SINGLE_ONE_CHAIN -DFCS_CHAINS=4 -DFCS_PREFETCH_DEPTH=1 -DFCS_LOAD_PRIO=0"),
    ("fcs_kernel.hip", "-DFCS_OLD_SINGLE -DFCS_NO_SINGLE -DFCS_WG_THREADS=768 -DFCS_FIXED_WG_THREADS=1024 "
                       "-DFCS_WIDE_SEGS=4"),
    ("fcs_kernel.hip", "-DFCS_NO_DMA -DFCS_DMA_WG_THREADS=768 -DFCS_DMA_CHAINS=4 -DFCS_DMA_AUX=0 "
                       "-DFCS_DMA_DYN_PCT=50 -DFCS_DMA_CHUNK_MAX=16"),
    ("fcs_kernel.hip", "-DFCS_DMA_PRIO -DFCS_DMA_EDGE_AUX=2 -DFCS_DMA_NO_TRIM -DFCS_DMA_ABL_NOALIGN "
                       "-DFCS_DMA_ABL_NOLDS"),
    ("fcs_kernel.hip", "-DFCS_NO_SEGIL -DFCS_SEGIL_TAIL_AUX=2 -DFCS_SEGIL_SKEW=0"),
    ("fcs_kernel.hip", "-DFCS_SEGIL_NOCRC -DFCS_SEGIL_ANY"),
    ("fcs_kernel.hip", "-DFCS_NO_WIDE"),
    ("fcs_kernel.hip", "-DFCS_WIDE_OLD_MASK"),
    ("fcs_kernel.hip", "-DFCS_WIDE_NO26 -DFCS_WIDE_NO30"),
    ("fcs_engine.cpp", "-DFCS_WIDE_MIN=1537"),
    ("fcs_engine.cpp", "-DFCS_WIDE_MID_MIN=0"),
    ("fcs_engine.cpp", "-DFCS_WIDE8_MIN=0 -DFCS_WIDE4_MIN=0"),
    ("fcs_engine.cpp", "-DFCS_SHORT_MAX=0 -DFCS_SHORT_WG_PER_CU=2"),
    ("fcs_kernel.hip", "-DFCS_SHORT_NO_PIPE"),
    ("fcs_kernel.hip", "-DFCS_WIDE_MID_WD_MIN=11"),
    ("fcs_engine.cpp", "-DFCS_WIDE_NO_PRE"),
    ("fcs_kernel.hip", "-DFCS_SEGIL_CMAX_ITEMS=100000"),
    ("fcs_engine.cpp", "-DFCS_SEGIL_ANY"),
    ("fcs_kernel.hip", "-DFCS_BLOCKED"),
    ("fcs_kernel.hip", "-DFCS_XCD -DFCS_NO_WAVE_SYNC"),
    ("fcs_kernel.hip", "-DFCS_FLAT_NOCRC -DFCS_FLAT_NO_SHORTCUTS -DFCS_FLAT_CHUNK_MAX=8 "
                       "-DFCS_FIXED_CHUNK_MAX=16 -DFCS_FIXED_DYN_PCT=50 -DFCS_MASK_ALL"),
    ("fcs_kernel.hip", "-DFCS_MASK_MINMAX -DFCS_ONE_NOBLOB -DFCS_ONE_NOARG"),
    ("fcs_kernel.hip", "-DFCS_STAMPS -DFCS_ST_AUX=0 -DFCS_ST_NOCRC"),
    ("fcs_kernel.hip", "-DFCS_ST_UNIT=1024 -DFCS_ST_CHAINS=2"),
    ("fcs_kernel.hip", "-DFCS_ST_ABL_NOCLOSE -DFCS_ST_ABL_NOSHIFT -DFCS_ST_NOSKEW"),
    ("fcs_kernel.hip", "-DFCS_ST_SKIPJ0 -DFCS_ST_PROBE_LDS=8 -DFCS_ST_PROBE_VALU=32"),
    ("fcs_kernel.hip", "-DFCS_ST_ALIGN16"),
    ("fcs_kernel.hip", "-DFCS_ST_EDGE_AUX=0"),
    ("fcs_kernel.hip", "-DFCS_SEGW_FORCE=26"),
    ("fcs_kernel.hip", "-DFCS_SEG_ITEM_WORDS=6"),
    ("inet_kernel.hip", "-DINET_EDGE_AUX=2 -DINET_ST_NOSUM"),
    ("fcs_engine.cpp", "-DFCS_FAULT_HOOK -DFCS_GRID_CUS=128 -DFCS_FLAT_DYN_MIN=1000 -DFCS_FIXED_DYN_MIN=8 "
                       "-DFCS_FIXED_FLAT_MAX=0 -DFCS_ZC_MAX_MB=16 -DFCS_NO_STREAM"),
    ("fcs_engine.cpp", "-DFCS_STAMPS -DFCS_HOST_TRACE -DFCS_PIPE_DEPTH=3"),
    ("fcs_txq.cpp", "-DFCS_TXQ_TSAN"),
    ("inet_kernel.hip", "-DFCS_NT"),
]


def _compile(tu, flags, out_dir, k):
    obj = os.path.join(out_dir, f"v{k}.o")
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c", "-o", obj,
           os.path.join(CSRC, tu)] + flags.split()
    r = subprocess.run(cmd, capture_output=True, text=True, cwd=out_dir)
    return tu, flags, r.returncode, r.stderr[-2000:]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_documented_variant_flags_compile():
    out_dir = tempfile.mkdtemp(prefix="fcs_variants_")
    try:
        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 1)) as ex:
            res = list(ex.map(lambda a: _compile(a[1][0], a[1][1], out_dir, a[0]), enumerate(VARIANTS)))
    finally:
        shutil.rmtree(out_dir, ignore_errors=True)
    failed = [(tu, fl, err) for tu, fl, rc, err in res if rc != 0]
    assert not failed, "\n\n".join(f"{tu} {fl}:\n{err}" for tu, fl, err in failed)


def test_every_switch_in_the_sources_is_covered():
    """A new FCS_* switch in the kernel or engine sources must be added to VARIANTS above."""
    import re
    used = set()
    for f in os.listdir(CSRC):
        src = open(os.path.join(CSRC, f)).read()
        used |= set(re.findall(r"#\s*(?:ifn?def|if defined\(|if)\s*\(?\s*(FCS_[A-Z0-9_]+)", src))
    covered = set(re.findall(r"FCS_[A-Z0-9_]+", " ".join(fl for _, fl in VARIANTS)))
    # include guards and constants that are not measurement switches
    exempt = {"FCS_LAUNCH"}
    missing = sorted(used - covered - exempt)
    assert not missing, f"switches not compiled by this test: {missing}"
