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
Inputs that are ill posed on purpose (the reference's ragged tol = 1e-6 fixture, the
Gram guard's floor cases) are marked "windowed": their tests assert the count against
the window (conftest.assert_iter_count), and only the oracle-in-window check runs here.
"""
import importlib
import math

import pytest

from oracle import aggregators as orc

MODULES = ["test_gpu_batched", "test_gpu_resident_batched", "test_gpu_weiszfeld",
           "test_gpu_panels", "test_gpu_sharded", "test_gpu_distributed", "test_gpu_fullsize",
           "test_gpu_c5_fullsize"]


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
        if flag != ["windowed"]:          # (windowed: the test asserts the window itself)
            assert w.width <= 1, (i, w, "tol on the fp32 movement floor: the count is rounding")
        opts = {"maxiter": maxiter, "tol": tol}
        if guess is not None:
            opts["guess"] = guess.float().clone()
        _, tr = orc.gm2(X.clone(), opts)
        if math.isfinite(tr.last_movement):
            assert w.early <= tr.iters <= w.late, (i, w, tr)
