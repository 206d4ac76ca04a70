"""The EMNIST AirComp call at its configured length, on the exchanges beyond one XCD
(VERDICT r5 item 2).

`EMNIST_Air_weight.py` runs the default aggregator `gm` (E:131-160 + OMA2 E:398-416) on
the EMNIST MLP, d = 48,670 (E:101), with maxiter 1000 (E:351), which `gm` always runs to
(its channel draw changes every iteration).  On the GPU that call takes the
single-problem register-resident kernel on a grid larger than one XCD, so its exchange is
not C2's one-XCD L2-kept gather (pinned by tests/test_gpu_c2_fullsize.py) but

* 50 x 48,670 (191 blocks): the XCD-hierarchical gather (member sums per XCD, then the 8
  group sums — a different reduction order from the flat gather);
* 50 x 20,000 (40 blocks): the split-scope one-hop exchange.

Both are AUTO's choice here (asserted through the result, not forced), pinned against
``oracle.gm`` (op for op E:131-160) fed the same Philox draws (``oracle.philox.gm_draws``)
for ALL 1000 iterations: relative L2 <= 1e-5, 1000 iterations.  Round 4 found drift that
only a full-length run exposed; these runs are the full length.

Inputs: the reference's caller (the guess = the current model p ~ N(0, 0.07^2), honest rows
p + N(0, (5e-4)^2), the last K/5 rows p + 2e-3 + N(0, (5e-3)^2); E:349-350).  There the
fp32 oracle and its fp64 run of the same draws agree to 7.6e-8 / 8.6e-8 after 1000
iterations (measured), so rounding is contracted, not amplified, and 1e-5 is a real bar.
"""
import pytest
import torch

from conftest import rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu

SEED = 20210518


def _caller(K, d, seed):
    g = torch.Generator().manual_seed(seed)
    p = 0.07 * torch.randn(d, generator=g)
    X = p + 5e-4 * torch.randn(K, d, generator=g)
    B = K // 5
    X[K - B:] = p + 2e-3 + 5e-3 * torch.randn(B, d, generator=g)
    return X, p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("K,d,exchange", [(50, 48_670, "xcd_hier"), (50, 20_000, "xcd_split")])
@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_emnist_gm_1000_iterations_vs_oracle(K, d, exchange, layout, monkeypatch):
    import byzantine_aircomp_amd as bz
    from oracle.philox import gm_draws
    for v in ("GMAGG_RES_HIER", "GMAGG_RES_SPLIT", "GMAGG_RES_XCD"):
        monkeypatch.delenv(v, raising=False)          # AUTO's own choice
    X, p = _caller(K, d, 1234 + d)
    opts = {"maxiter": 1000, "tol": 1e-5, "noise_var": 1e-2, "P_max": 1}
    Xd = X.cuda()
    if layout == "panels":
        Xd = bz.ClientPanels.from_rows(Xd)
    got = bz.gm(Xd, dict(opts, guess=p.cuda(), seed=SEED))
    torch.cuda.synchronize()
    res = bz.aggregators.last_result
    if layout == "rows":
        assert res.algo == "resident" and res.exchange == exchange, res
    assert res.iters == 1000 and not res.converged, res
    ref, tr = orc.gm(X, dict(opts, guess=p.clone()), draw=gm_draws(SEED, d))
    assert tr.iters == 1000
    err = rel_l2(got.cpu().numpy(), ref.numpy())
    print(f"emnist gm {K}x{d} {layout}: {res.algo} / {res.exchange}, rel L2 vs fp32 oracle {err:.3e}")
    assert torch.isfinite(got).all() and err <= 1e-5, err


@pytest.mark.timeout(600)
def test_emnist_gm2_call_vs_oracle():
    """The EMNIST `--agg gm2` call (E:162-184, maxiter 1000) on the same 191-block grid."""
    import byzantine_aircomp_amd as bz
    X, p = _caller(50, 48_670, 99)
    opts = {"maxiter": 1000, "tol": 1e-5}
    got = bz.gm2(X.cuda(), dict(opts, guess=p.cuda()))
    res = bz.aggregators.last_result
    assert res.algo == "resident" and res.exchange == "xcd_hier", res
    want, tr = orc.gm2(X, dict(opts, guess=p.clone()))
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= 1e-5
    assert abs(res.iters - tr.iters) <= 1, (res, tr)


def iteration_cases():
    """The +-1 input above, for tests/test_iteration_wellposed.py."""
    return [("emnist_gm2_50x48670", lambda: [(*_caller(50, 48_670, 99), 1000, 1e-5)])]
