"""AddressSanitizer + UBSan run of the host code that parses untrusted bytes (sanitizers on host code):
the FLAC decoder (csrc/flac.cpp) and the safetensors checkpoint reader (csrc/safetensors.cpp), built for the CPU by
tools/asan/Makefile with the mutation harness tools/asan/host_fuzz.cpp.  Well-formed inputs must decode to the
expected PCM / tensors (checksums computed here independently), and thousands of mutated ones (flipped bits,
truncations, inserted / deleted bytes, overwritten length fields) must all come back as a status -- any
out-of-bounds access, use-after-free, overflow or undefined shift aborts the harness.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import flac_writer as fw

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ASAN = os.path.join(ROOT, "tools", "asan")


def fnv(chunks, h=1469598103934665603):
    for b in chunks:
        for x in b:
            h = ((h ^ x) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.fixture(scope="module")
def harness():
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    r = subprocess.run(["make", "-C", ASAN], capture_output=True, text=True)
    if r.returncode != 0 and "sanitize" in r.stderr:
        pytest.skip("g++ without libasan / libubsan")
    assert r.returncode == 0, r.stderr[-2000:]
    return os.path.join(ASAN, "build", "host_fuzz")


def run(harness, files, mutations):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=24")
    r = subprocess.run([harness, "--mutations", str(mutations)] + [str(f) for f in files], capture_output=True,
                       text=True, env=env, timeout=600)
    assert r.returncode == 0 and "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, \
        (r.returncode, r.stderr[-4000:])
    lines = {}
    for ln in r.stdout.splitlines():
        if " status=" in ln:
            name, st, sm = ln.split()
            lines[name] = (int(st.split("=")[1]), int(sm.split("=")[1], 16))
    assert r.stdout.strip().endswith("ok")
    return lines


def test_flac_decoder_under_sanitizers(harness, tmp_path):
    rng = np.random.default_rng(3)
    files, want = [], {}
    for i, (C, bps, n) in enumerate([(1, 16, 5000), (2, 16, 3000), (1, 24, 2100), (2, 8, 777), (6, 12, 1500),
                                     (1, 16, 1)]):
        t = np.arange(n)
        pcm = np.stack([(np.sin(t * (0.01 + 0.003 * c)) * (2 ** (bps - 2)) +
                         rng.integers(-40, 40, n)).astype(np.int64) for c in range(C)])
        pcm = np.clip(pcm, -(1 << (bps - 1)), (1 << (bps - 1)) - 1)
        data = fw.encode(pcm, 16000, bps, block_sizes=[1024, 576], seed=i, variable=(i % 2 == 1), id3=(i == 2))
        p = tmp_path / f"c{i}.flac"
        p.write_bytes(data)
        files.append(p)
        want[str(p)] = fnv([pcm.astype(np.int32).tobytes()])
    got = run(harness, files, 400)
    for f in files:
        st, sm = got[str(f)]
        assert st == 0 and sm == want[str(f)], f


def test_safetensors_reader_under_sanitizers(harness, tmp_path):
    from safetensors.numpy import save_file
    rng = np.random.default_rng(4)
    files, want = [], {}
    cases = {
        "ok": {"a.weight": rng.standard_normal((3, 4, 5)).astype(np.float32), "b": np.zeros((0,), np.float32),
               "quantizer.x.embed_sum": rng.standard_normal((16, 8)).astype(np.float32)},
        "f16": {"a": rng.standard_normal((4,)).astype(np.float16)},
        "scalar": {"s": np.array(1.5, np.float32)},
    }
    for name, tensors in cases.items():
        p = tmp_path / f"{name}.safetensors"
        save_file(tensors, str(p), metadata={"format": "pt"})
        files.append(p)
        if all(v.dtype == np.float32 for v in tensors.values()):
            want[str(p)] = (0, fnv([k.encode() + np.ascontiguousarray(tensors[k]).tobytes() for k in sorted(tensors)]))
        else:
            want[str(p)] = (4, None)  # MIMI_ERR_WEIGHTS: the engine reads F32 checkpoints
    got = run(harness, files, 1500)
    for f in files:
        st, sm = got[str(f)]
        w = want[str(f)]
        assert st == w[0], (f, st)
        if w[1] is not None:
            assert sm == w[1], f


def test_config_json_reader_under_sanitizers(harness, tmp_path):
    """config.json (csrc/config_json.cpp) and 1500 mutations of it: a status every time, never an invalid access; the
    golden file reads as MIMI_OK."""
    golden = os.path.join(ROOT, "tests", "golden", "mimi_config.json")
    p = tmp_path / "config.json"
    p.write_bytes(open(golden, "rb").read())
    q = tmp_path / "nested.json"
    q.write_text('{"a": [[[{"b": "\\u00e9\\ud83d\\ude00"}]]], "upsampling_ratios": [8, 6, 5, 4], "frame_rate": 12.5}')
    got = run(harness, [p, q], 1500)
    assert got[str(p)][0] == 0 and got[str(q)][0] == 0
