"""ISA review of the built library (HIP ISA review), CPU only — tools/isa_review.py unbundles every linked
object's gfx950 code object and reads its metadata and disassembly.  Listed in .gpurunignore (it names scalar-store
mnemonics; it never runs on the GPU box)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_review  # noqa: E402


@pytest.fixture(scope="module")
def isa():
    if not os.path.exists(os.path.join(isa_review.LLVM, "clang-offload-bundler")):
        pytest.skip("ROCm LLVM tools not found")
    return isa_review.review()


def test_no_scalar_data_cache_writes(isa):
    """No kernel writes through the scalar data cache (scalar stores / atomics / cache write-back): the pool's rule."""
    assert isa["scalar_writes"] == [], isa["scalar_writes"][:5]


def test_headline_kernel_resources(isa):
    """k_fused<64,16,3,rk4> (BASELINE config 2): no scratch, at most 128 VGPRs (four waves per SIMD: the residency the
    fused kernel is designed for) and its products on the fp32 MFMA."""
    m = isa["kernels"][isa_review.HEADLINE]
    assert m["scratch"] == 0 and m["agpr"] == 0, m
    assert m["vgpr"] <= 128, m
    assert m["mfma"] >= 20, m


def test_every_kernel_has_metadata(isa):
    assert len(isa["kernels"]) > 100
    for name, m in isa["kernels"].items():
        assert {"vgpr", "sgpr", "scratch"} <= set(m), name
        assert m["vgpr"] <= 512, (name, m)  # (gfx950: .vgpr_count is the unified VGPR + AGPR allocation)


def test_no_waterfall_loops(isa):
    """Every buffer descriptor is built in SGPRs: a descriptor the compiler holds in VGPRs wraps each access in a
    waterfall loop (round 6: the adaptive solve's sample index reached its loop through LDS, 52 such loops in
    k_rows<32,2,0,1>, removed by readfirstlane'd bases)."""
    bad = {k: m["waterfalls"] for k, m in isa["kernels"].items() if m["waterfalls"]}
    assert not bad, bad
