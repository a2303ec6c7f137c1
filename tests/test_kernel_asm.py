"""Static checks of the compiled gfx950 device code (no GPU): no s_barrier is reached with an LDS write in flight
(tools/lds_barrier_scan.py -- the hipcc back-edge wait omission that made attention_band_h16_kernel racy)."""
import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def test_scanner_flags_a_missing_wait():
    import lds_barrier_scan as s
    racy = "_Zk:\n.LBB0_1:\n\ts_barrier\n\tds_read_b32 v1, v0\n\tds_write_b32 v0, v1\n\ts_branch .LBB0_1\n"
    safe = racy.replace("\ts_branch", "\ts_waitcnt lgkmcnt(0)\n\ts_branch")
    assert s.scan(racy) and not s.scan(safe)


@pytest.mark.skipif(not shutil.which("/opt/rocm/bin/hipcc"), reason="no hipcc")
def test_no_barrier_with_lds_write_in_flight(tmp_path):
    import lds_barrier_scan as s
    files = s.compile_all(str(tmp_path))
    bad = [b for f in files for b in s.scan(open(f).read())]
    assert not bad, bad[:5]
