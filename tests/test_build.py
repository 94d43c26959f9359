"""Build-time properties of libratis_hip (CPU; reads the compiler's resource-usage remarks that
ratis_amd/csrc/Makefile keeps under build/csrc/*.usage)."""
import glob
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _usage():
    files = sorted(glob.glob(os.path.join(ROOT, "build", "csrc", "*.usage")))
    if not files:
        pytest.skip("no build/csrc/*.usage (run __graft_entry__.build() first)")
    out = {}
    for f in files:
        name = None
        for line in open(f):
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
            m = re.search(r"ScratchSize \[bytes/lane\]: (\d+)", line)
            if m and name:
                out[(os.path.basename(f), name)] = int(m.group(1))
    return out


# Kernels pinned to 64 VGPRs (8 waves per SIMD, so a 1M-group launch is resident in one round)
# spill a few registers of their widest (joint-consensus) path.  Same-box A/B of the commit kernel
# at 8, 7 and 6 waves per SIMD (21, 4 and 0 spilled VGPRs): 4.53-4.62 TB/s for all three
# (profiles/r02/commit_waves/), so the pin stays; the allowance is a few dozen bytes per lane.
# crc_pack_kernel<true> (the read path's slot mode) runs at the 128-VGPR cap of its 1024-thread
# workgroup: a few per-lane constants are stored at kernel entry and reloaded once per 64-frame
# task (a few scratch loads per task, none in the step loop; gfx950 ISA checked, round 3).
SPILL_ALLOWED = {"commit_kernel_rank": 48, "leader_kernel": 48, "lease_kernel": 32, "crc_pack_kernel": 24}


def test_no_kernel_uses_scratch():
    """Every kernel keeps its state in registers / LDS: scratch (private memory in HBM) on a hot
    kernel means a spilled array or a by-value argument indexed per thread (the resident table's
    apply kernel once spilled its whole argument: 984 B per lane, 8x slower)."""
    u = _usage()
    assert u, "no kernels found in the usage remarks"
    bad = {}
    for (f, name), v in u.items():
        allowed = max([b for k, b in SPILL_ALLOWED.items() if k in name] or [0])
        if v > allowed:
            bad[(f, name)] = v
    assert not bad, bad
