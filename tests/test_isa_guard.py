"""CPU: the shipped library's gfx950 code holds no packed f32 FMA with a VGPR-pair second operand.

``v_pk_fma_f32 vD, vA, vB, vC`` (the form the SLP vectoriser makes from four scalar FMAs that share a broadcast
operand) gave different low-lane results when other kernels ran on the GPU at the same time (DESIGN.md §0 round 5,
tools/race_taps.py, profiles/r5z_*): ds_edge_fix_kernel's replicate-pad rows and conv0_kernel's tap.  The kernels
that would get it are built without SLP vectorisation (csrc/Makefile); this test keeps it out of the build."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tokenize-audio_amd", "mimi_hip", "libmimi_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
BAD = re.compile(r"\bv_pk_fma_f32\s+v\[\d+:\d+\],\s*[^,]+,\s*v\[\d+:\d+\]")


def _device_disassembly(tmp_path) -> str:
    if not os.path.exists(LIB):
        pytest.skip("libmimi_hip.so not built")
    if not os.path.exists(OBJDUMP):
        pytest.skip("llvm-objdump not installed")
    so = tmp_path / "lib.so"
    shutil.copy(LIB, so)
    subprocess.run([OBJDUMP, "--offloading", str(so)], cwd=tmp_path, check=True, capture_output=True)
    code = sorted(glob.glob(str(tmp_path / "lib.so.*gfx950*")))
    assert code, "no gfx950 code object in libmimi_hip.so"
    out = []
    for c in code:
        r = subprocess.run([OBJDUMP, "-d", c], check=True, capture_output=True, text=True)
        out.append(r.stdout)
    return "\n".join(out)


def test_no_packed_fma_with_vgpr_pair_operand(tmp_path):
    text = _device_disassembly(tmp_path)
    fn, bad = None, {}
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            fn = m.group(1)
        elif BAD.search(line):
            bad[fn] = bad.get(fn, 0) + 1
    assert not bad, f"packed f32 FMAs with a VGPR-pair operand in: {bad}"
    assert "mfma" in text  # (the disassembly is the real kernels')
