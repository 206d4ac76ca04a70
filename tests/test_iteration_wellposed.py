"""Every GPU test that asserts "the same iteration count +-1" (north_star) must ask a
well-posed question.  Runs on the CPU.

The reference stops at the first fp32 movement <= tol (M:180-183).  When tol sits on
the fp32 movement floor (~2^-24 ||g|| per ulp of the iterate), which of two roundings
happens to dip below tol decides the count, and a kernel that is right can land
several iterations away from the oracle (6 vs 8 at ||g|| ~ 8, tol 1e-6).
``oracle.gm2_count_window`` runs the exact (fp64) iteration and returns the range of
counts an fp32 implementation may legitimately stop at; the +-1 bar is well posed only
where that range is at most 2 wide.  Each GPU test module lists its +-1 inputs in
``iteration_cases()`` (built on the CPU with the same generators and parameters as the
test itself; device-filled inputs through oracle/philox.py's restatement of the fill),
so an ill-posed input fails here, in the container, instead of on the GPU box.

The fp32 oracle's own count must also fall inside the window (checks the window).
Flags: unmarked inputs must have a determined window at most 1 wide; "windowed" inputs
(the reference's fixtures, the Gram guard's accuracy case, the C4 floor-band case) a
determined window at most 2 wide (their tests assert the count against it,
conftest.assert_iter_count: at most 5 counts); "undetermined" inputs (tol at or below the
fp32 movement floor on purpose: the ragged tol = 1e-6 fixture, the guard's floor cases)
must really be undetermined, and their tests state their own bar (a slack with its
reason, or conftest.assert_floor_count).  Any other undetermined input fails here.
"""
import importlib
import math

import pytest

from conftest import MAX_WINDOW_WIDTH, assert_floor_count, assert_iter_count
from oracle import aggregators as orc

MODULES = ["test_gpu_batched", "test_gpu_resident_batched", "test_gpu_weiszfeld",
           "test_gpu_panels", "test_gpu_sharded", "test_gpu_distributed", "test_gpu_fullsize",
           "test_gpu_c5_fullsize", "test_gpu_resident_hier", "test_gpu_emnist_fullsize",
           "test_gpu_rows_pass"]


def _cases():
    out = []
    for name in MODULES:
        mod = importlib.import_module(name)
        if not hasattr(mod, "iteration_cases"):
            continue
        for cid, thunk in mod.iteration_cases():
            out.append(pytest.param(thunk, id=f"{name[9:]}:{cid}"))
    return out


@pytest.mark.parametrize("thunk", _cases())
def test_iteration_count_well_posed(thunk):
    for i, (X, guess, maxiter, tol, *flag) in enumerate(thunk()):
        X = X.float()
        w = orc.gm2_count_window(X, guess, maxiter, tol)
        if flag == ["undetermined"]:
            assert not w.determined, (i, w, "marked undetermined but the count is certain")
        else:
            assert w.determined, (i, w, "undetermined count window: tol at or below the fp32 "
                                        "movement floor, and the input is not marked")
            limit = MAX_WINDOW_WIDTH if flag == ["windowed"] else 1
            assert w.width <= limit, (i, w, "tol near the fp32 movement floor: the count is rounding")
        opts = {"maxiter": maxiter, "tol": tol}
        if guess is not None:
            opts["guess"] = guess.float().clone()
        _, tr = orc.gm2(X.clone(), opts)
        if math.isfinite(tr.last_movement):
            if w.determined:
                assert w.early <= tr.iters <= w.late, (i, w, tr)
            else:
                assert w.early <= tr.iters, (i, w, tr)


def test_floor_constant_shared_with_the_gram_guard():
    """The count window and the Gram guard's floor rule use ONE floor:
    oracle FLOOR_ULPS == gmagg_internal.h kFloorUlps (read from the source), and api.hip's
    guard computes its floor from that constant."""
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    csrc = os.path.join(root, "byzantine_aircomp_amd", "csrc")
    hdr = open(os.path.join(csrc, "gmagg_internal.h")).read()
    m = re.search(r"constexpr double kFloorUlps = ([0-9.]+);", hdr)
    assert m and float(m.group(1)) == orc.FLOOR_ULPS
    api = open(os.path.join(csrc, "api.hip")).read()
    assert "const double floor = kFloorUlps * u * gn;" in api


def test_assert_iter_count_bites():
    """The count assertions cannot pass vacuously: an undetermined window needs a stated
    slack, a determined window wider than 2 is refused, a floor count must be maxiter or
    an exact fixed point."""
    from types import SimpleNamespace
    und = orc.CountWindow(3, None, 100.0)
    with pytest.raises(AssertionError):
        assert_iter_count(900, 5, und)                      # no slack stated
    with pytest.raises(AssertionError):
        assert_iter_count(900, 5, und, 2, "reason")        # outside the slack
    assert_iter_count(6, 5, und, 1, "reason")
    with pytest.raises(AssertionError):
        assert_iter_count(7, 5, orc.CountWindow(4, 8, 1.0))  # 4 wide: refused
    assert_iter_count(7, 5, orc.CountWindow(5, 7, 1.0))
    with pytest.raises(AssertionError):
        assert_iter_count(9, 5, orc.CountWindow(5, 7, 1.0))
    assert_floor_count(SimpleNamespace(iters=30, last_movement=1e-4), 30, und)
    assert_floor_count(SimpleNamespace(iters=9, last_movement=0.0), 30, und)
    with pytest.raises(AssertionError):
        assert_floor_count(SimpleNamespace(iters=9, last_movement=1e-6), 30, und)
    with pytest.raises(AssertionError):
        assert_floor_count(SimpleNamespace(iters=2, last_movement=0.0), 30, und)
