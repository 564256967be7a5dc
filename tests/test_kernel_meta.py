"""Register / scratch budget of the built kernels (CPU: reads the gfx950 code object's
metadata out of libtdstep.so, no GPU).

A kernel that spills to scratch memory pays for it on every launch, not only where the
spill code runs: an A/B build whose step kernels carried 0.5-1 KB of scratch per lane
stepped 4.5x slower (profiles/r03/s4), and register allocation tips into spills on small
source changes.  So: no kernel of the library uses scratch, and the one-round small-batch
kernels at 10x10 keep the 8-waves-per-SIMD budget (<= 80 SGPRs, <= 64 VGPRs)."""
import os
import sys

import pytest

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(HERE, "scripts"))
import kernel_meta  # noqa: E402

TOOLS = all(os.path.exists(os.path.join(kernel_meta.LLVM, t)) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-readelf"))
pytestmark = pytest.mark.skipif(not (TOOLS and os.path.exists(kernel_meta.LIB)), reason="needs the built library and ROCm llvm tools")


@pytest.fixture(scope="module")
def meta():
    return kernel_meta.kernels()


def test_every_kernel_is_present(meta):
    for k in ("td_step_kernelILi10ELi0ELb0", "td_step_kernel_smallILi10ELi0ELb0", "td_step_kernel_small2ILi10ELi0ELb0",
              "td_step_kernelILi20ELi2ELb1", "td_step_kernel_small2ILi30ELi0ELb0", "td_refill_kernelILi10",
              "td_reset_kernelILi10", "td_autoreset_kernelILi10"):
        assert any(k in n for n in meta), k


def test_no_kernel_uses_scratch(meta):
    spilled = {n: r for n, r in meta.items() if r.get("scratch", 0) != 0}
    assert not spilled, spilled


def test_small_kernels_keep_eight_waves_at_10x10(meta):
    for n, r in meta.items():
        if ("td_step_kernel_smallILi10" in n or "td_step_kernel_small2ILi10" in n):
            assert r["sgpr"] <= 80 and r["vgpr"] <= 64, (n, r)
            assert r["lds"] * 32 <= 160 * 1024 * (2 if "small2" in n else 1), (n, r)  # 8 waves per SIMD fit LDS
