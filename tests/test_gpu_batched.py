"""Batched independent aggregations (row f1, BASELINE C5) vs single calls and the oracle."""
import pytest
import torch

from conftest import rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu


def _problems(P, K, d, seed):
    g = torch.Generator().manual_seed(seed)
    p = 0.07 * torch.randn(P, 1, d, generator=g)
    X = p + 5e-4 * torch.randn(P, K, d, generator=g)
    for i in range(P):
        B = (0, 5, 10)[i % 3] if K >= 20 else 0
        if B:
            X[i, K - B:] = p[i] + 5e-3 * torch.randn(B, d, generator=g) + 2e-3
    return X, p[:, 0, :]


ORACLE_SHAPES = [(1, 50, 7852), (7, 50, 10_000), (12, 17, 333), (33, 64, 4096)]


@pytest.mark.parametrize("P,K,d", ORACLE_SHAPES)
def test_gm2_batched_matches_oracle(P, K, d):
    from byzantine_aircomp_amd.batched import gm2_batched
    X, p = _problems(P, K, d, seed=P * 100 + K)
    out, res = gm2_batched(X.cuda(), {"maxiter": 1000, "guess": p.cuda()})
    for i in range(P):
        want, tr = orc.gm2(X[i].clone(), {"maxiter": 1000, "tol": 1e-5, "guess": p[i].clone()})
        assert rel_l2(out[i].cpu().numpy(), want.numpy()) <= 1e-5
        assert abs(res[i].iters - tr.iters) <= 1


def test_gm_batched_equals_single_calls():
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.batched import SEED_STRIDE, gm_batched
    P, K, d = 6, 50, 20_000
    X, p = _problems(P, K, d, seed=5)
    X, p = X.cuda(), p.cuda()
    opts = {"maxiter": 30, "tol": 1e-5, "noise_var": 1e-2, "seed": 99}
    out, res = gm_batched(X, dict(opts, guess=p))
    for i in range(P):
        single = bz.gm(X[i], dict(opts, guess=p[i], seed=(99 + i * SEED_STRIDE) % 2 ** 64))
        assert rel_l2(out[i].cpu().numpy(), single.cpu().numpy()) <= 1e-5
        assert res[i].iters == 30


def _mixed_problems():
    X, p = _problems(5, 30, 2048, seed=8)
    # a harder problem (converges later), seeded: the round-3 version drew it from the
    # global generator, so the input depended on what ran before in the process
    X[2] = torch.randn(30, 2048, generator=torch.Generator().manual_seed(88))
    return X, p


def test_batched_mixed_convergence():
    """Problems converge at different iterations; each stops at its own tol test.
    tol 1e-5, not 1e-6: problem 2's ||g|| ~ 8 puts the fp32 movement floor
    (~4 * 2^-24 * ||g|| = 2e-6) above 1e-6, where the count measures rounding
    (oracle.gm2_count_window; tests/test_iteration_wellposed.py checks every +-1 input)."""
    from byzantine_aircomp_amd.batched import gm2_batched
    X, p = _mixed_problems()
    out, res = gm2_batched(X.cuda(), {"maxiter": 1000, "guess": p.cuda(), "tol": 1e-5})
    iters = [r.iters for r in res]
    assert len(set(iters)) > 1
    for i in range(5):
        want, tr = orc.gm2(X[i].clone(), {"maxiter": 1000, "tol": 1e-5, "guess": p[i].clone()})
        assert rel_l2(out[i].cpu().numpy(), want.numpy()) <= 1e-5
        assert abs(iters[i] - tr.iters) <= 1


@pytest.mark.parametrize("P,K,d", [(5, 50, 10_000), (3, 7, 333)])
def test_oma_batched_equals_single_calls(P, K, d):
    """C5 in the reference's literal `--agg gm2 --var v` reading (M:351-353): the
    batched OMA pre-noise of problem p is bit-identical to OMA(X[p]) with seed
    + p * SEED_STRIDE (float4 path at d % 4 == 0, scalar path otherwise)."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.batched import SEED_STRIDE, oma_batched
    X, _ = _problems(P, K, d, seed=17)
    X = X.cuda()
    batched = oma_batched(X.clone(), 1e-2, seed=123)
    for i in range(P):
        single = X[i].clone()
        bz.OMA(single, 1e-2, seed=(123 + i * SEED_STRIDE) % 2 ** 64)
        assert torch.equal(batched[i], single), i
    assert not torch.equal(batched, X)


def test_c5_prenoise_reading_matches_oracle():
    """OMA pre-noise then gm2, batched, vs the oracle gm2 on the same noisy problems."""
    from byzantine_aircomp_amd.batched import gm2_batched, oma_batched
    P, K, d = 4, 50, 8192
    X, p = _problems(P, K, d, seed=23)
    Xn = oma_batched(X.cuda(), 1e-3, seed=7)
    out, res = gm2_batched(Xn, {"maxiter": 1000, "guess": p.cuda()})
    Xh = Xn.cpu()
    for i in range(P):
        want, tr = orc.gm2(Xh[i].clone(), {"maxiter": 1000, "tol": 1e-5, "guess": p[i].clone()})
        assert rel_l2(out[i].cpu().numpy(), want.numpy()) <= 1e-5
        assert abs(res[i].iters - tr.iters) <= 1


PANEL_SHAPES = [(50, 7850), (50, 4099), (200, 3000), (7, 513), (20, 4096), (100, 2048)]


def _panel_problems(K, d):
    P = 5
    g = torch.Generator().manual_seed(K * 3 + d)
    X = 0.05 * torch.randn(P, K, d, generator=g)
    X[:, K - K // 5:] += 0.25
    g0 = 0.01 * torch.randn(P, d, generator=g)
    return X, g0


@pytest.mark.parametrize("K,d", PANEL_SHAPES)
@pytest.mark.parametrize("agg", ["gm2", "gm"])
def test_batched_panels_match_rows(K, d, agg):
    """ProblemPanels (every problem in the panel layout) vs the row-major batched call:
    bit-identical where both run the same tile (d % 4 == 0, K outside 32 < K <= 64 and
    128 < K <= 256),
    equal to rounding otherwise; batched OMA identical draw for draw."""
    from byzantine_aircomp_amd.batched import ProblemPanels, gm2_batched, gm_batched, oma_batched
    X, g0 = _panel_problems(K, d)
    P = X.shape[0]
    X, g0 = X.cuda(), g0.cuda()
    Pn = ProblemPanels.from_rows(X)
    assert torch.equal(Pn.to_rows(), X)
    oma_batched(X, 1e-2, seed=5)
    oma_batched(Pn, 1e-2, seed=5)
    assert torch.equal(Pn.to_rows(), X)
    f = gm2_batched if agg == "gm2" else gm_batched
    # gm never converges and its iterate grows without bound on this data: 8 iterations
    # keep the rounding differences of the other-tile cases from being amplified
    # (the streaming batched path on both layouts: the register-resident kernel takes the
    # panels but not a contiguous [P, K, d] with d % 4 != 0; its own layout test is in
    # test_gpu_resident_batched.py)
    opts = {"maxiter": 40 if agg == "gm2" else 8, "tol": 1e-5, "guess": g0, "algo": "stream"}
    if agg == "gm":
        opts.update(noise_var=1e-2, seed=7)
    a, ra = f(X, dict(opts))
    b, rb = f(Pn, dict(opts))
    if d % 4 == 0 and not (32 < K <= 64 or 128 < K <= 256):
        assert torch.equal(a, b)
        assert [r.iters for r in ra] == [r.iters for r in rb]
    else:
        # (gm amplifies the other tile's summation order over its iterations: the gm
        # parity bar of test_gpu_weiszfeld.py, 1e-5)
        tol = 1e-6 if agg == "gm2" else 1e-5
        for p in range(P):
            assert rel_l2(b[p].cpu().numpy(), a[p].cpu().numpy()) <= tol
            assert abs(ra[p].iters - rb[p].iters) <= 1


def test_batched_gm_rows_staged_as_panels():
    """Row-major batched AirComp gm over >= 64 passes (P*K*d >= 2^24) is packed once into
    the context's panel buffer (api.hip gm_weiszfeld_batched_f32): bit-identical to the
    ProblemPanels call, and each problem equal to rounding to a single row-major
    `gm(..., algo="stream")` call with the problem's seed (not staged)."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.batched import SEED_STRIDE, ProblemPanels, gm_batched
    P, K, d = 4, 300, 16_384
    g = torch.Generator().manual_seed(31)
    X = (0.05 * torch.randn(P, K, d, generator=g)).cuda()
    X[:, : K // 10] += 0.3
    g0 = (0.01 * torch.randn(P, d, generator=g)).cuda()
    opts = {"maxiter": 64, "tol": 1e-5, "noise_var": 1e-2, "seed": 11, "guess": g0}
    a, ra = gm_batched(X, dict(opts))
    b, rb = gm_batched(ProblemPanels.from_rows(X), dict(opts))
    assert torch.equal(a, b)
    assert [r.iters for r in ra] == [r.iters for r in rb] == [64] * P
    for i in range(P):
        single = bz.gm(X[i], dict(opts, guess=g0[i], seed=(11 + i * SEED_STRIDE) % 2 ** 64,
                                  algo="stream"))
        assert rel_l2(a[i].cpu().numpy(), single.cpu().numpy()) <= 1e-5


def iteration_cases():
    """Every input above whose iteration count is asserted +-1, built on the CPU
    (tests/test_iteration_wellposed.py): (id, thunk -> [(X, guess, maxiter, tol), ...])."""
    from oracle.philox import oma_philox
    SEED_STRIDE = 0x9E3779B97F4A7C15
    cases = []
    for P, K, d in ORACLE_SHAPES:
        def t(P=P, K=K, d=d):
            X, p = _problems(P, K, d, seed=P * 100 + K)
            return [(X[i], p[i], 1000, 1e-5) for i in range(P)]
        cases.append((f"oracle_{P}x{K}x{d}", t))

    def mixed():
        X, p = _mixed_problems()
        return [(X[i], p[i], 1000, 1e-5) for i in range(5)]
    cases.append(("mixed_convergence", mixed))

    def prenoise():
        X, p = _problems(4, 50, 8192, seed=23)
        return [(torch.from_numpy(oma_philox(X[i].numpy(), 1e-3, (7 + i * SEED_STRIDE) % 2 ** 64))
                 .float(), p[i], 1000, 1e-5) for i in range(4)]
    cases.append(("c5_prenoise", prenoise))
    for K, d in PANEL_SHAPES:
        def t(K=K, d=d):
            X, g0 = _panel_problems(K, d)
            return [(X[i], g0[i], 40, 1e-5) for i in range(X.shape[0])]
        cases.append((f"panels_{K}x{d}", t))
    return cases
