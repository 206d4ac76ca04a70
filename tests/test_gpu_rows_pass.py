"""The 32-wave row-major kernel (rows_pass.hip, round 6): the gm2 STEP / INIT passes on the
reference's own [K, d] stack at 512 < K <= 1024 (the layout `flatten_list` builds, M:206-209),
against the oracle and against the generic streaming tile it replaces.

* gm2 (M:162-184) through AUTO on row-major inputs at the kernel's edges — K = 513 (the
  first K it takes), 1000 (C3's), 1024 (its full tile: every row group in use); d from one
  partial 32-column chunk (20) to many; a padded row stride (ldx > d) — against
  ``oracle.gm2``: rel L2 <= 1e-5 and the iteration count +-1 (windows checked by
  tests/test_iteration_wellposed.py);
* the same call with GMAGG_ROWS_LEAN=0 (the generic tile): the same iteration count and the
  aggregate equal to rounding (rel L2 <= 1e-6), not bit for bit — the two kernels sum a
  column's rows in different orders, which is how the test knows the 32-wave kernel ran;
* inputs it does not take (K = 512, d % 4 != 0, AirComp gm) keep their results.
"""
import pytest
import torch

from conftest import rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu


def _recipe(K, d, seed, ldx=None):
    g = torch.Generator().manual_seed(seed)
    B = K // 5
    X = 0.05 * torch.randn(K, d, generator=g)
    X[K - B:] = 0.25 + 0.5 * torch.randn(B, d, generator=g)
    g0 = 0.01 * torch.randn(d, generator=g)
    if ldx is not None:
        buf = torch.zeros(K, ldx)
        buf[:, :d] = X
        return buf, g0
    return X, g0


CASES = [(513, 4096, None), (1000, 20, None), (1000, 20_000, None), (1024, 12_288, None),
         (1000, 8192, 8200), (700, 65_540, None)]


@pytest.mark.parametrize("K,d,ldx", CASES)
def test_rows_pass_vs_oracle_and_generic(K, d, ldx, monkeypatch):
    import byzantine_aircomp_amd as bz
    Xs, g0 = _recipe(K, d, K + d, ldx)
    X = Xs[:, :d]                                  # a strided view when ldx is padded
    opts = {"maxiter": 1000, "tol": 1e-5}
    want, tr = orc.gm2(X.contiguous(), dict(opts, guess=g0.clone()))
    Xd = Xs.cuda()[:, :d]
    monkeypatch.delenv("GMAGG_ROWS_LEAN", raising=False)
    a = bz.gm2(Xd, dict(opts, guess=g0.cuda()))
    ra = bz.aggregators.last_result
    assert ra.algo == "stream", ra
    assert rel_l2(a.cpu().numpy(), want.numpy()) <= 1e-5
    assert abs(ra.iters - tr.iters) <= 1, (ra, tr)
    monkeypatch.setenv("GMAGG_ROWS_LEAN", "0")
    b = bz.gm2(Xd, dict(opts, guess=g0.cuda()))
    rb = bz.aggregators.last_result
    assert rb.iters == ra.iters, (ra, rb)
    assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-6
    if d >= 4096:
        assert not torch.equal(a, b)               # a different kernel summed the rows


@pytest.mark.parametrize("K,d,agg", [(512, 4096, "gm2"), (1000, 4097, "gm2"), (1000, 4096, "gm")])
def test_rows_pass_not_taken(K, d, agg, monkeypatch):
    """Shapes and modes outside the kernel: the generic tile's results, bit for bit."""
    import byzantine_aircomp_amd as bz
    X, g0 = _recipe(K, d, 3)
    opts = {"maxiter": 50, "tol": 1e-5, "guess": g0.cuda(), "algo": "stream"}
    if agg == "gm":
        opts.update(noise_var=1e-2, seed=5)
    fn = getattr(bz, agg)
    monkeypatch.delenv("GMAGG_ROWS_LEAN", raising=False)
    a = fn(X.cuda(), dict(opts))
    monkeypatch.setenv("GMAGG_ROWS_LEAN", "0")
    b = fn(X.cuda(), dict(opts))
    assert torch.equal(a, b)


def iteration_cases():
    """The +-1 inputs above, for tests/test_iteration_wellposed.py."""
    def case(K, d, ldx):
        Xs, g0 = _recipe(K, d, K + d, ldx)
        return [(Xs[:, :d].contiguous(), g0, 1000, 1e-5)]
    return [(f"rows_pass_{K}x{d}", lambda K=K, d=d, ldx=ldx: case(K, d, ldx)) for K, d, ldx in CASES]


@pytest.mark.parametrize("val", [float("nan"), float("inf"), -float("inf")])
@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_rows_pass_special_values(val, layout):
    """One NaN / +-inf element (NaN is never <= tol, so the call runs to
    maxiter): the reference's iterate turns all-NaN — an infinite row gets weight 0 and
    0 * inf = NaN in its column, then every distance is NaN — and so does the 32-wave rows
    kernel's (and the panel tile's), after the same maxiter iterations."""
    import byzantine_aircomp_amd as bz
    X, g0 = _recipe(600, 4096, 11)
    X[17, 123] = val
    opts = {"maxiter": 7, "tol": 1e-5, "guess": g0.clone()}
    want, tr = orc.gm2(X.clone(), dict(opts))
    Xd = X.cuda() if layout == "rows" else bz.ClientPanels.from_rows(X.cuda())
    out = bz.gm2(Xd, dict(opts, guess=g0.cuda()))
    r = bz.aggregators.last_result
    assert r.algo == "stream" and r.iters == tr.iters == 7, (r, tr)
    assert torch.equal(torch.isnan(out.cpu()), torch.isnan(want))
    assert torch.isnan(out).all()
