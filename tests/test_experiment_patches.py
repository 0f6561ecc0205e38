"""The measured-and-not-kept kernel experiments live as patches under tools/k5_exp/ (DESIGN.md §4,
profiles/r9_ab.txt), rebuilt on demand by tools/build_variant.sh (PATCH=...).  Each must still apply
to the current sources, or its numbers could no longer be reproduced.  CPU only: a dry run of
`patch`, nothing is built."""
import glob
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PATCHES = sorted(glob.glob(os.path.join(ROOT, "tools", "k5_exp", "*.patch")))


@pytest.mark.skipif(shutil.which("patch") is None, reason="no patch(1) here")
@pytest.mark.parametrize("path", PATCHES, ids=[os.path.basename(p) for p in PATCHES])
def test_experiment_patch_applies(path):
    r = subprocess.run(["patch", "--dry-run", "-s", "-f", "-p1", "-d", ROOT, "-i", path],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


def test_experiment_patches_present():
    names = {os.path.basename(p) for p in PATCHES}
    assert {"k5s_slice.patch", "k5_dma_swz.patch", "k5_scan_server.patch", "k5_steal.patch",
            "k1_filter.patch"} <= names
