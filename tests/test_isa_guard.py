"""CPU: the shipped library's gfx950 code holds no packed f32 instruction at all.

Packed f32 (``v_pk_fma_f32``, ``v_pk_mul_f32``, ``v_pk_add_f32``, ``v_pk_mov_b32``) gave different low-lane results
while other kernels ran on the GPU at the same time (DESIGN.md "Packed f32", tools/race_taps.py, tools/pk_probe.hip,
profiles/r5z_*, r6*_pk_probe*).  Round 5 kept out only the one operand form that was caught (a VGPR-pair broadcast
FMA); every device object is now compiled with the packed-fp32-ops target feature off (csrc/Makefile), and this test
rejects the whole instruction class in every kernel, whatever the operand form or the instruction that makes it."""
import glob
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tokenize-audio_amd", "mimi_hip", "libmimi_hip.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
PACKED_F32 = re.compile(r"\bv_pk_(?:fma_f32|mul_f32|add_f32|mov_b32)\b")


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


def packed_f32_by_kernel(text: str) -> dict:
    fn, bad = None, {}
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            fn = m.group(1)
        elif PACKED_F32.search(line):
            bad[fn] = bad.get(fn, 0) + 1
    return bad


def test_guard_pattern_covers_every_operand_form():
    # the forms round 5's library held (SGPR-pair, broadcast op_sel, negated, plain VGPR pairs) all match
    for line in ("v_pk_fma_f32 v[2:3], v[60:61], v[56:57], v[2:3] op_sel_hi:[1,0,1]",
                 "v_pk_fma_f32 v[4:5], v[6:7], s[2:3], v[4:5]",
                 "v_pk_mul_f32 v[0:1], v[2:3], s[4:5] op_sel_hi:[1,0]",
                 "v_pk_add_f32 v[0:1], v[2:3], v[4:5] neg_lo:[0,1] neg_hi:[0,1]",
                 "v_pk_mov_b32 v[0:1], v[2:3], v[4:5] op_sel:[0,1]"):
        assert PACKED_F32.search(line), line
    for line in ("v_pk_fma_f16 v0, v1, v2, v3", "v_pk_mul_f16 v0, v1, v2", "v_fma_f32 v0, v1, v2, v3"):
        assert not PACKED_F32.search(line), line


def test_no_packed_f32_in_any_kernel(tmp_path):
    text = _device_disassembly(tmp_path)
    bad = packed_f32_by_kernel(text)
    assert not bad, f"packed f32 instructions in: {bad}"
    assert "mfma" in text  # (the disassembly is the real kernels')
