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

# Fixtures whose count window is undetermined (tol at or below the fp32 movement floor):
# the bar each one's count is held to, and the measured reason (tools/dbg/iter_counts.py,
# profiles/r5s1_iter_counts.txt)
FIXTURE_SLACK = {
    "gm2_ragged_K7_d777": (1, "tol 1e-6 sits below the 2-ulp fp32 movement floor of ||g|| ~ 10 "
                              "(1.2e-6): the reference stops at 10, every GPU path at 9"),
}


def assert_fixture_count(got, name):
    """The count bar of gm2 golden fixture `name` against the reference's own count."""
    meta, _ = golden_case(name)
    slack, why = FIXTURE_SLACK.get(name, (None, None))
    assert_iter_count(got, meta["iters"], fixture_window(name), slack, why)


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


MAX_WINDOW_WIDTH = 2       # [early - 1, late + 1]: at most 5 accepted counts


def assert_iter_count(got, want, window=None, slack=None, why=None):
    """north_star's "same iteration count +-1" where the question is well posed.

    * No window, or a window at most 1 wide: |got - want| <= 1.
    * A determined window 2 wide (tol near the fp32 movement floor of the input,
      oracle.gm2_count_window): the count lies in [early - 1, late + 1] (5 counts); a wider
      determined window is refused — the input belongs to the undetermined case's bar.
    * An undetermined window (tol at or below the floor: no count is certain): the test
      states its own bar — ``slack`` (<= 2) against ``want`` (the reference's or the fp32
      oracle's count) and ``why``, the measured reason it holds."""
    if window is not None and not window.determined:
        assert slack is not None and why, ("undetermined count window: the test must state a "
                                           "slack and its reason", window)
        assert 0 <= slack <= 2, slack
        assert abs(got - want) <= slack, (got, want, slack, why, window)
        return
    if window is None or window.width <= 1:
        assert abs(got - want) <= 1, (got, want, window)
        return
    assert window.width <= MAX_WINDOW_WIDTH, ("count window too wide for a count bar", window)
    assert window.early - 1 <= got <= window.late + 1, (got, want, window)


def assert_floor_count(res, maxiter, window):
    """The count bar where tol sits far below the fp32 movement floor (an undetermined
    window whose floor is several times tol, e.g. ||g|| ~ 500-1500 at tol 1e-5): an fp32
    Weiszfeld's movement never falls below tol by rounding there, so it runs to maxiter
    (the reference does) — unless its iterate lands on an exact fixed point of its own
    fp32 arithmetic (movement exactly 0), which can only happen once the exact iteration
    has converged, i.e. at a count >= window.early.  Exactly these two outcomes pass."""
    assert window is not None and not window.determined, window
    if res.iters == maxiter:
        return
    assert res.last_movement == 0.0 and window.early <= res.iters < maxiter, (res, window)
