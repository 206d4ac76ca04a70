"""The single-problem register-resident kernel on grids larger than one XCD (round 5,
VERDICT r4 item 6): the EMNIST MLP (E:101, d = 48,670: 96 blocks) and 50 x 20,000 (40
blocks) gather XCD by XCD — each block's partials L2-kept for its XCD's leader, the 8 per-XCD
sums exchanged agent-scope (resident.hip, `a.hier`) — instead of every block polling every
other block across the fabric.

* against the oracle: gm2 (M:162-184) rel L2 <= 1e-5 and iterations +-1; gm (M:131-160)
  with Philox draws against oracle.gm fed the same draws (oracle.philox.gm_draws), 200
  iterations, rel L2 <= 1e-5;
* against the flat gather (GMAGG_RES_HIER=0) on the same inputs: the reduction order
  differs (group sums first), so the results agree at the rounding level (rel L2 <= 1e-6
  for gm2, 1e-5 for 200 gm iterations) with the same iteration count;
* the hierarchical result is reproducible bit for bit (the grouping is fixed by the
  block index, not by where the blocks land).

The parity tests force the hierarchical gather on every grid beyond one XCD
(GMAGG_RES_HIER=2); AUTO takes it only where it measured faster (test_hier_default_choice).
"""
import pytest
import torch

from conftest import rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu

SHAPES = [(50, 48_670), (50, 20_000), (40, 48_670)]


def _caller(K, d, seed):
    g = torch.Generator().manual_seed(seed)
    p = 0.07 * torch.randn(d, generator=g)
    X = p + 5e-4 * torch.randn(K, d, generator=g)
    B = K // 5
    X[K - B:] = p + 2e-3 + 5e-3 * torch.randn(B, d, generator=g)
    return X, p


@pytest.mark.parametrize("K,d", SHAPES)
def test_hier_gm2_vs_oracle_and_flat(K, d, monkeypatch):
    import byzantine_aircomp_amd as bz
    monkeypatch.setenv("GMAGG_RES_HIER", "2")          # every grid beyond one XCD
    X, p = _caller(K, d, K * 7 + d)
    opts = {"maxiter": 1000, "tol": 1e-5}
    want, tr = orc.gm2(X.clone(), dict(opts, guess=p.clone()))
    Xd, pd = X.cuda(), p.cuda()
    a = bz.gm2(Xd, dict(opts, guess=pd))
    ra = bz.aggregators.last_result
    assert ra.algo == "resident" and ra.exchange == "xcd_hier", ra
    assert rel_l2(a.cpu().numpy(), want.numpy()) <= 1e-5
    assert abs(ra.iters - tr.iters) <= 1, (ra, tr)
    b = bz.gm2(Xd, dict(opts, guess=pd))
    assert torch.equal(a, b)                               # reproducible
    monkeypatch.setenv("GMAGG_RES_HIER", "0")
    monkeypatch.setenv("GMAGG_RES_SPLIT", "0")          # the flat gather
    f = bz.gm2(Xd, dict(opts, guess=pd))
    rf = bz.aggregators.last_result
    assert rf.algo == "resident" and rf.exchange == "agent", rf
    assert rf.iters == ra.iters
    assert rel_l2(a.cpu().numpy(), f.cpu().numpy()) <= 1e-6


@pytest.mark.parametrize("K,d", SHAPES[:2])
def test_hier_gm_philox_vs_oracle_and_flat(K, d, monkeypatch):
    import byzantine_aircomp_amd as bz
    from oracle.philox import gm_draws
    monkeypatch.setenv("GMAGG_RES_HIER", "2")
    X, p = _caller(K, d, K * 11 + d)
    it, seed = 200, 31337
    opts = {"maxiter": it, "tol": 1e-5, "noise_var": 1e-2, "P_max": 1}
    got = bz.gm(X.cuda(), dict(opts, guess=p.cuda(), seed=seed))
    res = bz.aggregators.last_result
    assert res.algo == "resident" and res.exchange == "xcd_hier" and res.iters == it, res
    ref, tr = orc.gm(X, dict(opts, guess=p.clone()), draw=gm_draws(seed, d))
    assert tr.iters == it
    assert rel_l2(got.cpu().numpy(), ref.numpy()) <= 1e-5
    monkeypatch.setenv("GMAGG_RES_HIER", "0")
    monkeypatch.setenv("GMAGG_RES_SPLIT", "0")          # the flat gather
    flat = bz.gm(X.cuda(), dict(opts, guess=p.cuda(), seed=seed))
    assert bz.aggregators.last_result.exchange == "agent"
    assert rel_l2(got.cpu().numpy(), flat.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("K,d", [(50, 20_000), (40, 48_670)])
def test_split_scope_equals_flat(K, d, monkeypatch):
    """The split-scope exchange (GMAGG_RES_SPLIT=1: every granule published agent-scope and
    L2-kept, each reader polling its own XCD's blocks from the L2-kept copy) carries the
    same values in the same order as the flat gather: bit-identical results, gm2 and gm."""
    import byzantine_aircomp_amd as bz
    X, p = _caller(K, d, 77)
    Xd, pd = X.cuda(), p.cuda()
    monkeypatch.setenv("GMAGG_RES_HIER", "0")
    for agg, opts in (("gm2", {"maxiter": 1000, "tol": 1e-5}),
                      ("gm", {"maxiter": 100, "tol": 1e-5, "noise_var": 1e-4, "seed": 3})):
        outs = {}
        for sp in ("1", "0"):
            monkeypatch.setenv("GMAGG_RES_SPLIT", sp)
            outs[sp] = (getattr(bz, agg)(Xd, dict(opts, guess=pd)), bz.aggregators.last_result)
        (a, ra), (b, rb) = outs["1"], outs["0"]
        assert ra.algo == rb.algo == "resident" and ra.iters == rb.iters, (ra, rb)
        assert (ra.exchange, rb.exchange) == ("xcd_split", "agent"), (ra, rb)
        assert bool(torch.isfinite(a).all()) and torch.equal(a, b)


def test_hier_default_choice():
    """AUTO takes the hierarchical gather where it measured faster (>= 90 blocks at
    K > 32: the EMNIST MLP's 50 x 48,670, 191 blocks of 256 columns since round 5's block
    rule, 96 of 512 before) and the split-scope one-hop exchange on
    the other grids beyond one XCD (50 x 20,000: 40 blocks); both exist for the 8-wave tile
    (32 < K <= 64) only, so K = 10 gathers flat (profiles/r5s1_resident_*_ab.jsonl)."""
    import byzantine_aircomp_amd as bz
    for (K, d), want in (((50, 48_670), "xcd_hier"), ((50, 20_000), "xcd_split"),
                         ((10, 48_670), "agent"), ((50, 7850), "xcd_local")):
        X, p = _caller(K, d, 3)
        bz.gm2(X.cuda(), {"maxiter": 20, "tol": 1e-5, "guess": p.cuda()})
        r = bz.aggregators.last_result
        assert r.algo == "resident" and r.exchange == want, (K, d, r)


def test_hier_checkin_failure_streams(monkeypatch):
    """A hierarchical grid that fails its co-residency check-in (GMAGG_RES_CHECKIN_FAIL=1:
    one slot nobody writes) streams within one 100 ms check-in, and the result equals the
    streaming path's."""
    import time

    import byzantine_aircomp_amd as bz
    bz.aggregators.close_all()                       # a fresh context (no skip state)
    X, p = _caller(50, 48_670, 5)
    Xd, opts = X.cuda(), {"maxiter": 1000, "tol": 1e-5, "guess": p.cuda()}
    want = bz.gm2(Xd, dict(opts, algo="stream"))
    monkeypatch.setenv("GMAGG_RES_CHECKIN_FAIL", "1")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    got = bz.gm2(Xd, dict(opts))
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    monkeypatch.delenv("GMAGG_RES_CHECKIN_FAIL")
    assert bz.aggregators.last_result.algo == "stream"
    assert dt < 1.5, dt
    assert torch.equal(got, want)
    bz.aggregators.close_all()


def iteration_cases():
    """The +-1 inputs above, for tests/test_iteration_wellposed.py."""
    cases = []
    for K, d in SHAPES:
        cases.append((f"hier_{K}x{d}", lambda K=K, d=d: [(*_caller(K, d, K * 7 + d), 1000, 1e-5)]))
    cases.append(("hier_batched_q5", lambda: [(*_caller(50, 100_000, 905), 1000, 1e-5)]))
    return cases


@pytest.mark.parametrize("mode", ["1"])
@pytest.mark.parametrize("agg", ["gm2", "gm"])
def test_batched_hier_vs_flat(agg, mode, monkeypatch):
    """The batched resident kernel (C5's) with its groups gathering XCD by XCD (mode 1:
    sub-group leaders, then the <= 3 sub-group sums; an A/B knob, off by default) against
    the flat group gather (GMAGG_RB_HIER=0, the default): the same problems, results equal
    at the rounding level
    (gm2: rel L2 <= 1e-6 and the same counts; gm, 300 iterations at var 1e-3 on the caller
    recipe: <= 1e-5), and problem 5 against the oracle."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.batched import SEED_STRIDE, ProblemPanels, gm2_batched, gm_batched
    from oracle.philox import gm_draws
    P, K, d = 12, 50, 100_000
    Xs, ps = zip(*[_caller(K, d, 900 + q) for q in range(P)])
    X = torch.stack(Xs).cuda()
    g0 = torch.stack(ps).cuda()
    Pn = ProblemPanels.from_rows(X)
    it, seed = 300, 4242
    opts = {"maxiter": 1000 if agg == "gm2" else it, "tol": 1e-5, "guess": g0}
    if agg == "gm":
        opts.update(noise_var=1e-3, seed=seed)
    run = gm2_batched if agg == "gm2" else gm_batched
    outs = {}
    for h in (mode, "0"):
        monkeypatch.setenv("GMAGG_RB_HIER", h)
        out, res = run(Pn, dict(opts))
        assert all(r.algo == "resident" for r in res), res[0]
        outs[h] = (out.cpu(), res)
    (a, ra), (b, rb) = outs[mode], outs["0"]
    assert (ra[0].exchange == "xcd_hier") == (mode == "1") and rb[0].exchange != "xcd_hier"
    assert [r.iters for r in ra] == [r.iters for r in rb]
    assert rel_l2(a.numpy(), b.numpy()) <= (1e-6 if agg == "gm2" else 1e-5)
    q = 5
    if agg == "gm2":
        want, tr = orc.gm2(X[q].cpu(), {"maxiter": 1000, "tol": 1e-5, "guess": g0[q].cpu()})
        assert abs(ra[q].iters - tr.iters) <= 1
    else:
        want, tr = orc.gm(X[q].cpu(), {"maxiter": it, "tol": 1e-5, "noise_var": 1e-3, "P_max": 1,
                                       "guess": g0[q].cpu()},
                          draw=gm_draws((seed + q * SEED_STRIDE) % 2 ** 64, d))
    assert rel_l2(a[q].numpy(), want.numpy()) <= 1e-5
