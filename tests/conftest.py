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
