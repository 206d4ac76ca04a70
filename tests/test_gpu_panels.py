"""The panel layout (ClientPanels, GM_LAYOUT_PANELS) on the GPU.

Same values, same chunks, same reduction order as the row-major call with the
float4 tile (d % 4 == 0), so the aggregate, the iteration count and the last
movement must be BIT-identical to gm2 / gm on the [K, d] tensor — which the
row-major tests pin to the reference (test_gpu_weiszfeld.py); other d within
rounding, and so is row-major gm2 at 512 < K <= 1024, which runs the 32-wave rows
kernel (rows_pass.hip, round 6); plus the reference's golden vectors directly.
"""
import numpy as np
import pytest
import torch

from conftest import assert_fixture_count, golden_case, golden_names, rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu


def bz():
    import byzantine_aircomp_amd as m
    return m


def _data_cpu(K, d, seed, byz=0.2):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(K, d, generator=g) * 0.05
    nb = int(K * byz)
    if nb:
        X[K - nb:] = torch.randn(nb, d, generator=g) * 0.5 + 0.25
    g0 = torch.randn(d, generator=g) * 0.01
    return X, g0


def _data(K, d, seed, byz=0.2):
    X, g0 = _data_cpu(K, d, seed, byz)
    return X.cuda(), g0.cuda()


BIT_SHAPES = [(1, 5), (7, 1), (50, 7850), (50, 4099), (129, 1000), (300, 2051), (1000, 4096),
              (1000, 70001), (1500, 3000)]


@pytest.mark.parametrize("K,d", BIT_SHAPES)
@pytest.mark.parametrize("agg", ["gm2", "gm"])
def test_panels_bit_identical_to_rows(K, d, agg):
    X, g0 = _data(K, d, seed=K * 7 + d)
    P = bz().ClientPanels.from_rows(X)
    assert torch.equal(P.to_rows(), X)
    opts = {"maxiter": 50, "tol": 1e-5, "guess": g0, "algo": "stream"}
    if agg == "gm":
        opts.update(noise_var=1e-2, seed=99)
    f = getattr(bz(), agg)
    a = f(X, dict(opts))
    ra = bz().aggregators.last_result
    b = f(P, dict(opts))
    rb = bz().aggregators.last_result
    assert rb.algo == "stream"
    if d % 4 == 0 and not (32 < K <= 64 or 128 < K <= 256):
        # the row-major call runs the same float4 tile: same chunks, same order (at
        # 32 < K <= 64 and 128 < K <= 256 panels have a tile of their own, api.hip pick_cfg;
        # row-major gm2 at 512 < K <= 1024 runs the 32-wave rows kernel, rows_pass.hip,
        # whose column sums take another order: equal to rounding)
        assert (ra.iters, ra.converged) == (rb.iters, rb.converged)
        if agg == "gm2" and 512 < K <= 1024:
            assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-6
            assert abs(ra.last_movement - rb.last_movement) <= 1e-3 * rb.last_movement
        else:
            assert torch.equal(a, b)
            assert ra.last_movement == rb.last_movement or (np.isnan(ra.last_movement)
                                                            and np.isnan(rb.last_movement))
    else:
        # row-major runs another tile here (float2/float1 for d % 4 != 0, or the
        # wider INIT tile): other summation grouping, equal to rounding
        assert rel_l2(b.cpu().numpy(), a.cpu().numpy()) <= 1e-6
        assert abs(ra.iters - rb.iters) <= 1


@pytest.mark.parametrize("name", golden_names("gm2"))
def test_panels_match_reference_gm2(name):
    meta, arr = golden_case(name)
    o = dict(meta["options"])
    if o.get("maxiter", 200) == 0:
        pytest.skip("maxiter 0 returns the guess object (covered by the row-major test)")
    if meta.get("guess_supplied"):
        o["guess"] = torch.from_numpy(arr["guess"].copy()).cuda()
    P = bz().ClientPanels.from_rows(torch.from_numpy(arr["X"].copy()).cuda())
    out = bz().gm2(P, o)
    res = bz().aggregators.last_result
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= 1e-5
    assert_fixture_count(res.iters, name)


def test_panels_store_rows_and_default_guess():
    K, d = 24, 1236                           # d % 4 == 0, K <= 32: the same float4 tile
    X, _ = _data(K, d, seed=5)
    P = bz().ClientPanels(K, d)
    for k in range(K):
        P.store(k, X[k])
    assert torch.equal(P.to_rows(), X)
    assert torch.equal(P.row(3), X[3])
    # (AUTO takes a register-resident kernel on either layout: pin the streaming pass)
    a = bz().gm2(X, {"maxiter": 20, "guess": X.mean(dim=0), "algo": "stream"})
    b = bz().gm2(P, {"maxiter": 20, "guess": X.mean(dim=0), "algo": "stream"})
    assert torch.equal(a, b)
    c = bz().gm2(P, {"maxiter": 20})          # guess = column mean of the panels
    assert bz().aggregators.last_result.algo == "resident"
    assert rel_l2(c.cpu().numpy(), a.cpu().numpy()) <= 1e-6


def test_panels_reject_non_streaming_algos():
    """Panels run the streaming pass, (gm2, K <= 256) the f16 Gram or a resident kernel
    (K <= 64 on a grid that fits one XCD: C2's; else K <= 52: the batched one); the other
    algorithms, the f32 Gram, Gram for AirComp gm or K > 256, and "resident" at K = 65
    raise.  At K = 64 and a small d "resident" runs C2's kernel."""
    X, g0 = _data(64, 512, seed=1)
    P = bz().ClientPanels.from_rows(X)
    for algo in ("twopass", "gram_f32"):
        with pytest.raises(RuntimeError):
            bz().gm2(P, {"maxiter": 5, "guess": g0, "algo": algo})
    bz().gm2(P, {"maxiter": 5, "guess": g0, "algo": "resident"})
    assert bz().aggregators.last_result.algo == "resident"
    X65, g65 = _data(65, 512, seed=1)
    with pytest.raises(RuntimeError):
        bz().gm2(bz().ClientPanels.from_rows(X65), {"maxiter": 5, "guess": g65, "algo": "resident"})
    with pytest.raises(RuntimeError):
        bz().gm(P, {"maxiter": 5, "guess": g0, "algo": "gram", "noise_var": 1e-2})
    X2, g2 = _data(300, 512, seed=2)
    with pytest.raises(RuntimeError):
        bz().gm2(bz().ClientPanels.from_rows(X2), {"maxiter": 5, "guess": g2, "algo": "gram"})
    # gm2 at K <= 256: explicit Gram on panels is supported (guarded)
    out = bz().gm2(P, {"maxiter": 5, "guess": g0, "algo": "gram"})
    assert bz().aggregators.last_result.algo in ("gram", "stream") and out.shape == (512,)


@pytest.mark.parametrize("K,d", [(50, 7850), (1000, 4099), (300, 257)])
def test_oma_philox_on_panels_equals_rows(K, d):
    """OMA's Philox draws are keyed by (client, global column): the panel kernel adds
    exactly the noise the row-major kernel adds, and leaves the padding at zero."""
    X, _ = _data(K, d, seed=11)
    P = bz().ClientPanels.from_rows(X)
    bz().OMA(X, 1e-2, seed=42)
    bz().OMA(P, 1e-2, seed=42)
    assert torch.equal(P.to_rows(), X)
    if d % P.W:
        assert torch.count_nonzero(P.data[-1, :, d % P.W:]) == 0


@pytest.mark.parametrize("K,d,W,offset", [(1000, 4099, None, 0), (3, 37, None, 0), (50, 7850, None, 1),
                                          (7, 100, 6, 0), (600, 8192, None, 0)])
def test_rows_to_panels_kernel_matches_layout(K, d, W, offset):
    """gm_rows_to_panels_f32 (pack.hip) writes exactly the panel image of the rows:
    float4 and scalar paths (misaligned rows, W not a multiple of 4), ragged last
    panel with its padding left zero."""
    from byzantine_aircomp_amd.panels import ClientPanels
    g = torch.Generator().manual_seed(K + d)
    buf = torch.randn(K * d + offset, generator=g).cuda()
    X = buf[offset:].view(K, d)
    P = ClientPanels(K, d, W=W)
    P.copy_rows_(X)
    torch.cuda.synchronize()
    Wd = P.W
    npan = -(-d // Wd)
    ref = torch.zeros(K, npan * Wd)
    ref[:, :d] = X.cpu()
    ref = ref.view(K, npan, Wd).transpose(0, 1)
    assert torch.equal(P.data.cpu(), ref)
    assert torch.equal(P.to_rows().cpu(), X.cpu())


GRAM_SHAPES = [(256, 1 << 18), (200, (1 << 18) + 4160), (64, (1 << 18) + 36), (33, 300_000),
               (1, 1 << 18)]


def _gram_data(K, d):
    g = torch.Generator().manual_seed(K + d)
    X = 0.05 * torch.randn(K, d, generator=g)
    B = K // 5
    if B:
        X[K - B:] = 0.25 + 0.5 * torch.randn(B, d, generator=g)
    return X, 0.01 * torch.randn(d, generator=g)


@pytest.mark.parametrize("K,d", GRAM_SHAPES)
def test_gram_on_panels_matches_rows_and_stream(K, d):
    """gm2 at K <= 256 on ClientPanels: AUTO takes the scaled-f16 Gram straight from
    the panel layout (W-column panels, 64-column stages), guarded; it agrees with
    the row-major Gram and with the streaming path."""
    m = bz()
    X, g0 = _gram_data(K, d)
    X, g0 = X.cuda(), g0.cuda()
    P = m.ClientPanels.from_rows(X)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": g0}
    a = m.gm2(P, dict(opts))
    ra = m.aggregators.last_result
    assert ra.algo == "gram" and ra.guard == "accepted" and ra.gram_kind == "f16_split"
    b = m.gm2(X, dict(opts, algo="gram"))
    rb = m.aggregators.last_result
    assert rb.algo == "gram" and ra.iters == rb.iters
    assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-6
    c = m.gm2(P, dict(opts, algo="stream"))
    assert abs(m.aggregators.last_result.iters - ra.iters) <= 1
    assert rel_l2(a.cpu().numpy(), c.cpu().numpy()) <= 1e-5


def test_gram_on_panels_overflow_falls_back_to_stream():
    """An element past the f16 headroom on panels: no bf16 panel kernel, so the
    call ends on the streaming path (guard 'rejected') and still matches."""
    m = bz()
    g = torch.Generator().manual_seed(5)
    K, d = 64, 1 << 18
    X = 0.05 * torch.randn(K, d, generator=g)
    X[K - 12:] += 0.25
    X[5, 200_000] = 1e6
    p = torch.zeros(d)
    want, tr = orc.gm2(X.clone(), {"maxiter": 1000, "tol": 1e-5, "guess": p})
    P = m.ClientPanels.from_rows(X.cuda())
    got = m.gm2(P, {"maxiter": 1000, "tol": 1e-5, "guess": p.cuda()})
    res = m.aggregators.last_result
    assert res.algo == "stream" and res.guard == "rejected"
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= 1e-5
    assert abs(res.iters - tr.iters) <= 1


SINGLE_SHAPES = [(50, 7850, "gm2"), (1, 5, "gm2"), (20, 100_003, "gm2"), (30, 8192, "gm"),
                 (52, 4096, "gm2")]


@pytest.mark.parametrize("K,d,agg", SINGLE_SHAPES)
def test_single_panels_call_runs_resident(K, d, agg):
    """One ClientPanels problem at K <= 52 (gm: K <= 50), AUTO: the batched register-resident
    kernel with P = 1 (X read once for all iterations) instead of one streaming pass per
    iteration; it matches the oracle (gm2) or the streaming path on the same Philox draws
    (gm, a fixed number of iterations)."""
    X, g0 = _data(K, d, seed=K + d)
    P = bz().ClientPanels.from_rows(X)
    f = getattr(bz(), agg)
    if agg == "gm2":
        got = f(P, {"maxiter": 1000, "tol": 1e-5, "guess": g0})
        res = bz().aggregators.last_result
        assert res.algo == "resident"
        want, tr = orc.gm2(X.cpu(), {"maxiter": 1000, "tol": 1e-5, "guess": g0.cpu()})
        assert rel_l2(got.cpu().numpy(), want.numpy()) <= 1e-5
        assert abs(res.iters - tr.iters) <= 1
    else:
        opts = {"maxiter": 25, "tol": 1e-5, "guess": g0, "noise_var": 1e-2, "seed": 9}
        got = f(P, dict(opts))
        res = bz().aggregators.last_result
        assert res.algo == "resident" and res.iters == 25
        ref = f(P, dict(opts, algo="stream"))
        assert bz().aggregators.last_result.algo == "stream"
        assert rel_l2(got.cpu().numpy(), ref.cpu().numpy()) <= 1e-4


RES_PANEL_SHAPES = [(50, 7850, "gm2"), (50, 7850, "gm"), (30, 4098, "gm"), (20, 4098, "gm2"),
                    (52, 2050, "gm2")]


@pytest.mark.parametrize("K,d,agg", RES_PANEL_SHAPES)
def test_single_panels_resident_matches_rows(K, d, agg):
    """A single ClientPanels problem whose resident grid fits one XCD runs C2's kernel
    (resident.hip) on the panels with its rows tile, V = 2 columns per lane inside one
    panel (api.hip).  At d % 4 == 2 the row-major call runs that same tile (float2 rows), so
    both read the same columns in the same lanes and agree bit for bit, iterations too."""
    X, g0 = _data(K, d, seed=K * 11 + d)
    P = bz().ClientPanels.from_rows(X)
    opts = {"maxiter": 200, "tol": 1e-5, "guess": g0}
    if agg == "gm":
        opts.update(maxiter=100, noise_var=1e-2, seed=3)
    f = getattr(bz(), agg)
    a = f(X, dict(opts))
    ra = bz().aggregators.last_result
    b = f(P, dict(opts))
    rb = bz().aggregators.last_result
    assert ra.algo == "resident" and rb.algo == "resident"
    assert torch.equal(a, b)
    assert (ra.iters, ra.converged) == (rb.iters, rb.converged)


def iteration_cases():
    """The +-1 inputs above, on the CPU (tests/test_iteration_wellposed.py); the golden
    fixtures are listed by test_gpu_weiszfeld.py, the 1e6-spike input equals its own."""
    cases = []
    for K, d in BIT_SHAPES:
        cases.append((f"bit_{K}x{d}", lambda K=K, d=d: [(*_data_cpu(K, d, K * 7 + d), 50, 1e-5)]))
    for K, d in GRAM_SHAPES:
        cases.append((f"gram_{K}x{d}", lambda K=K, d=d: [(*_gram_data(K, d), 1000, 1e-5)]))
    for K, d, agg in SINGLE_SHAPES:
        if agg == "gm2":
            cases.append((f"single_{K}x{d}",
                          lambda K=K, d=d: [(*_data_cpu(K, d, K + d), 1000, 1e-5)]))
    return cases
