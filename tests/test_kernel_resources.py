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
# SGPR spills (into VGPR lanes via v_writelane / v_readlane: no scratch, but VALU and registers in
# the kernel's loop): none in the streaming / fused hot kernels; the rest capped at what the
# round-6 build has, so a regression shows (round 5: the wide conv's 57-73 -> 16-20 by CD_OPQ).
SGPR_SPILL_CAP = {"k_fused4": 0, "k_fused": 0, "k_r2h_stream": 0, "k_h2r_stream": 0,
                  "k_r2h_down": 0, "k_hexconv_stream": 0, "k_hexconv_mfma_bf16d": 20,
                  "k_hexconv_mfma_bf16": 12, "k_tri_up": 16, "k_hexresize_down": 25,
                  "k_pyr_stream": 24}


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


def _family(sym):
    import re
    m = re.search(r"(k_\w+?)(I|E|P)", sym)
    return m.group(1) if m else sym


@pytest.mark.skipif(not os.path.exists(LIB) or shutil.which("objcopy") is None
                    or not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-readobj"),
                    reason="needs the built library and the ROCm LLVM tools")
def test_hot_kernels_sgpr_spills_capped():
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from kernel_resources import resources
    res = resources(LIB)
    seen, bad = set(), {}
    for k, (_, ss, _) in res.items():
        fam = _family(k)
        if fam in SGPR_SPILL_CAP:
            seen.add(fam)
            if ss > SGPR_SPILL_CAP[fam]:
                bad[k] = (ss, SGPR_SPILL_CAP[fam])
    assert seen == set(SGPR_SPILL_CAP), set(SGPR_SPILL_CAP) - seen
    assert not bad, bad
