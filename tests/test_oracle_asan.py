"""The CPU restatement under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY 5:
the CPU-side safety net of the -ffp-contract=off fp64 oracle).  `make -C oracle asan`
builds hg_oracle.c with oracle/selftest.c (edge shapes, every conv mode, fp64 adjoint
identities of the resamplers and of HexConv2d) and runs it; any sanitizer report or
failed identity exits non-zero."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_selftest_under_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "selftest: ok" in r.stdout
