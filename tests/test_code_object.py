"""The shipped gfx950 code object: no kernel spills VGPRs or uses scratch memory, and every
kernel's register count leaves room for the waves its workgroup size asks for.

VERDICT r2 asked for `vgpr_spill_count` 0. Scratch is as bad: in round 3 the generic fixed-length
kernel kept its 120-byte work dispenser in scratch memory (a pointer to it that could be null), and
a scratch load in a loop waits with `vmcnt`, together with the frame loads in flight. CPU only:
the code object metadata comes from `llvm-objdump --offloading` and `llvm-readelf --notes`.
"""
import os
import re
import shutil
import subprocess
import tempfile

import pytest

import nstack_amd as na

LLVM = "/opt/rocm/lib/llvm/bin"


def _kernels(lib_path):
    tmp = tempfile.mkdtemp(prefix="fcs_co_")
    try:
        lib = os.path.join(tmp, os.path.basename(lib_path))
        shutil.copy(lib_path, lib)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", lib], capture_output=True, cwd=tmp, check=True)
        out = []
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" not in f or "gfx950" not in f:
                continue
            notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", os.path.join(tmp, f)], capture_output=True,
                                   text=True, check=True).stdout
            for block in notes.split("  - .agpr_count:")[1:]:
                field = lambda k: re.search(rf"\.{k}:\s+(\S+)", block).group(1)
                out.append({"name": field("name"), "vgpr": int(field("vgpr_count")),
                            "vgpr_spill": int(field("vgpr_spill_count")),
                            "sgpr_spill": int(field("sgpr_spill_count")),
                            "scratch": int(field("private_segment_fixed_size")),
                            "wg": int(field("max_flat_workgroup_size"))})
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-readelf"), reason="ROCm LLVM tools not installed")
def test_no_spills_no_scratch_and_registers_fit_the_workgroup():
    ks = _kernels(na.LIB_PATH)
    names = {k["name"] for k in ks}
    for want in ("fcs_dma_kernel", "fcs_segil_kernel", "fcs_segw_kernel", "fcs_stream_kernel", "fcs_flat_kernel", "fcs_one_kernel",
                 "inet_flat_kernel"):
        assert any(want in n for n in names), want
    bad = [k for k in ks if k["vgpr_spill"] or k["scratch"]]
    assert not bad, bad
    # one workgroup per CU (the LDS tables): wg / 256 waves per SIMD, 512 VGPRs per SIMD lane
    tight = [k for k in ks if k["wg"] > 256 and k["vgpr"] > 512 // (k["wg"] // 256)]
    assert not tight, tight


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/llvm-readelf"), reason="ROCm LLVM tools not installed")
def test_baseline_kernels_spill_no_sgprs():
    """The kernels of the BASELINE configs (the LDS-DMA kernel: 1518 B; the arena stream: IMIX; the
    interleaved segments of either window: jumbo) and the wide windows keep every scalar in SGPRs: a spilled SGPR costs
    a v_writelane / v_readlane pair per use (the segment kernel had 10)."""
    hot = ("fcs_dma_kernel", "fcs_segil_kernel", "fcs_segw_kernel", "fcs_stream_kernel", "fcs_wide_kernel")
    ks = [k for k in _kernels(na.LIB_PATH) if any(h in k["name"] for h in hot)]
    assert len(ks) >= 40
    bad = [(k["name"], k["sgpr_spill"]) for k in ks if k["sgpr_spill"]]
    assert not bad, bad
