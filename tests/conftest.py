import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU) and libgmagg.so")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


def golden_manifest():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def golden_case(name):
    for c in golden_manifest()["cases"]:
        if c["name"] == name:
            return c, dict(np.load(os.path.join(GOLDEN, c["file"])))
    raise KeyError(name)


def golden_names(func):
    return [c["name"] for c in golden_manifest()["cases"] if c["func"] == func]


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


_WINDOWS = {}


def fixture_window(name):
    """oracle.gm2_count_window of a gm2 golden fixture (cached)."""
    if name not in _WINDOWS:
        import torch
        from oracle import aggregators as orc
        meta, arr = golden_case(name)
        o = meta["options"]
        guess = torch.from_numpy(arr["guess"].copy()) if meta.get("guess_supplied") else None
        _WINDOWS[name] = orc.gm2_count_window(torch.from_numpy(arr["X"].copy()), guess,
                                              o.get("maxiter", 200), o.get("tol", 1e-5))
    return _WINDOWS[name]


def assert_iter_count(got, want, window=None):
    """north_star's "same iteration count +-1" where the question is well posed.

    Where tol sits on the fp32 movement floor of the input (``window.width > 1``,
    oracle.gm2_count_window), the reference's own count is decided by rounding; the bar
    there is that the count lies in the window of counts an fp32 Weiszfeld may
    legitimately stop at (widened by 1 on each side, as +-1 is)."""
    if window is None or window.width <= 1:
        assert abs(got - want) <= 1, (got, want, window)
    else:
        assert window.early - 1 <= got <= window.late + 1, (got, want, window)
