import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "tokenize-audio_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


_PARITY_LOG = []


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


@pytest.fixture(scope="session")
def parity_log():
    """Parity tests append {test, codes, exact, chain_flips, max_flip_margin, ...}; the session writes them to
    gpurun_out/parity_report.json (copied into profiles/ with the round's evidence)."""
    return _PARITY_LOG


def pytest_sessionfinish(session, exitstatus):
    if not _PARITY_LOG:
        return
    import json
    out = os.path.join(ROOT, "gpurun_out")
    try:
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, "parity_report.json"), "w") as f:
            json.dump({"exitstatus": int(exitstatus), "records": _PARITY_LOG}, f, indent=1)
    except OSError:
        pass


def assert_codes_in_range(codes, ncodes=2048):
    """Every code a test sees is a codebook index: [0, ncodes)."""
    import numpy as np
    a = codes.detach().cpu().numpy() if hasattr(codes, "detach") else np.asarray(codes)
    if a.size:
        lo, hi = int(a.min()), int(a.max())
        assert 0 <= lo and hi < ncodes, f"code outside [0, {ncodes - 1}]: min {lo}, max {hi}"


@pytest.fixture(scope="session", autouse=True)
def _codes_range_guard():
    """Session-wide: every code array the engine returns to a test through the model (full encodes, async tickets of
    full encodes, the quantizer alone) or the drop-in wrapper (trimmed per item, ragged included) is checked to lie in
    [0, 2047] -- a code the engine could only produce by returning an unfinished RVQ."""
    try:
        from mimi_hip import encoder as enc_mod
        from mimi_hip import model as model_mod
    except Exception:  # (the package does not import: the tests that need it fail on their own)
        yield
        return
    M, E, T = model_mod.MimiHipModel, enc_mod.MimiEncoder, model_mod.EncodeTicket
    saved = []

    def wrap(cls, name, check):
        orig = getattr(cls, name)
        saved.append((cls, name, orig))

        def f(self, *a, **k):
            out = orig(self, *a, **k)
            check(self, out)
            return out
        f.__wrapped__ = orig
        setattr(cls, name, f)

    wrap(M, "encode", lambda self, out: assert_codes_in_range(out[0]))
    wrap(M, "encode_int32", lambda self, out: assert_codes_in_range(out))
    wrap(M, "encode_host", lambda self, out: assert_codes_in_range(out))
    wrap(M, "quantize", lambda self, out: assert_codes_in_range(out))
    # tickets of full (non-ragged) encodes: a ragged output's frames past an item's own are unspecified
    orig_async = M.encode_async

    def enc_async(self, *a, **k):
        t = orig_async(self, *a, **k)
        t._range_check = True
        return t
    saved.append((M, "encode_async", orig_async))
    M.encode_async = enc_async
    orig_wait = T.wait

    def wait(self):
        out = orig_wait(self)
        if getattr(self, "_range_check", False):
            assert_codes_in_range(out)
        return out
    saved.append((T, "wait", orig_wait))
    T.wait = wait
    wrap(E, "encode_audio_chunk", lambda self, out: assert_codes_in_range(out))
    wrap(E, "encode_audio_batch", lambda self, out: [assert_codes_in_range(c) for c in out])
    wrap(E, "encode_audio_chunks", lambda self, out: [assert_codes_in_range(c) for c in out])
    yield
    for cls, name, orig in reversed(saved):
        setattr(cls, name, orig)


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    with np.load(os.path.join(GOLDEN, "golden.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    with open(os.path.join(GOLDEN, "golden_meta.json")) as f:
        meta = json.load(f)
    return arrays, meta


@pytest.fixture(scope="session")
def state_dict():
    from mimi_hip import synthetic
    return synthetic.make_state_dict(seed=0)
