"""Device checks of the wave primitives behind the scans' top-k sorts and cross-workgroup merges
(pf_device.h lane_xor32 — DPP quad permutes, row mirrors / rotations, the gfx950 permlane16/32
swaps — wave_sort64 and wave_min64) against a host sort: tools/probe/lane_xor.hip, built by
__graft_entry__.build() (tools/Makefile)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = os.path.join(ROOT, "tools", "probe", "lane_xor")


@pytest.mark.gpu
def test_lane_xor_sort_min_primitives():
    assert os.path.exists(PROBE), "tools/probe/lane_xor not built (run __graft_entry__.build())"
    r = subprocess.run([PROBE], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


def test_lane_xor_probe_source_present():
    assert os.path.exists(PROBE + ".hip")
