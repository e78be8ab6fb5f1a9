"""No hot-path kernel of the built library uses scratch or spills VGPRs (CPU check of the code
object metadata, tools/kernel_resources.py).  Round 5: a run-time array index put 128 B per
lane of every nearest k_tri_up into scratch, and a 4-wave register cap spilled k_hexresize_down
(DESIGN.md §8c); both were invisible in the source.  The general (non-streaming) kernels listed
below keep their scratch: run-time indexed tap arrays off the hot path, and fp64 pooling."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hybrid-grid-for-hexagonal-and-rectangular-image-processing_amd", "HyGrid",
                   "_lib", "libhygrid_hip.so")
GENERAL = ("k_resample_nearest", "k_resample_bwd", "k_homography", "k_pool_")


@pytest.mark.skipif(not os.path.exists(LIB) or shutil.which("objcopy") is None
                    or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readobj"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_hot_kernels_have_no_scratch_or_vgpr_spills():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import resources
    res = resources(LIB)
    assert len(res) > 500, "the library's kernels were not found"
    bad = {k: v for k, v in res.items() if (v[0] or v[2]) and not any(g in k for g in GENERAL)}
    assert not bad, bad
    hot = [k for k in res if any(h in k for h in ("k_fused4", "k_tri_up", "k_hexresize_down",
                                                   "k_r2h_stream", "k_h2r_stream", "k_fused"))]
    assert hot and all(res[k][0] == 0 and res[k][2] == 0 for k in hot)
