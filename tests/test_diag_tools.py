"""The diagnostic recipes DESIGN.md cites stay reproducible on the current sources:
every scripts/*.patch (timing-only or stamped builds, applied to a copy by
scripts/build_fast.sh SRCDIR=...) still applies, and the stand-alone measurement
kernels (scripts/lds_gather.hip, scripts/pool_sweep.hip) still compile for gfx950.
CPU only: nothing here runs on a GPU."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCHES = sorted(glob.glob(os.path.join(ROOT, "scripts", "*.patch")))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(shutil.which("patch") is None, reason="no patch(1)")
@pytest.mark.parametrize("path", PATCHES, ids=[os.path.basename(p) for p in PATCHES])
def test_patch_applies(path):
    r = subprocess.run(["patch", "--dry-run", "-p1", "-i", path], cwd=ROOT, capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    out = r.stdout.lower()
    assert "failed" not in out and "ignored" not in out, r.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="no hipcc")
@pytest.mark.parametrize("src", ["lds_gather.hip", "pool_sweep.hip"])
def test_measurement_kernel_compiles(src):
    r = subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-fsyntax-only",
                        os.path.join(ROOT, "scripts", src)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
