"""The resident table's tile layout (ratis_amd/csrc/rh_internal.h, tile::pair_off / elem_off):
every column element of every width lies inside its tile and the int64 columns cover their
region exactly once, for the shipped column layout and the row-group records the RH_TABLE_GROUP
knob selects.  Host code only: hipcc compiles it here without a GPU."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("group", [128, 16, 8, 2])
def test_tile_layout_is_a_bijection(tmp_path, group):
    exe = tmp_path / f"layout_{group}"
    subprocess.run([HIPCC, "-std=c++17", f"-DRH_TABLE_GROUP={group}", "-I", os.path.join(ROOT, "ratis_amd", "csrc"),
                    "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "layout_check", "layout_check.cpp"),
                    "-o", str(exe)], check=True, capture_output=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    assert out.returncode == 0 and "violations: 0" in out.stdout, out.stdout
