"""GPU parity of the HIP Weiszfeld aggregators against the reference's golden
vectors and the CPU oracle.

Bar (BASELINE.json north_star): relative L2 <= 1e-5 in fp32 on the aggregate
and the same iteration count +-1.  OMA with the reference's own draws must be
bit-exact.  All calls go through the C ABI (libgmagg.so) via the drop-in
module.
"""
import math

import numpy as np
import pytest
import torch

from conftest import (FIXTURE_SLACK, assert_fixture_count, assert_floor_count, assert_iter_count,
                      golden_case, golden_names, rel_l2)
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu
TOL = 1e-5          # relative L2 on the aggregate (north_star)
ITER_SLACK = 1      # iteration count +-1 (north_star)


def bz():
    import byzantine_aircomp_amd as m
    return m


def _opts(meta, arr, dev="cuda"):
    o = dict(meta["options"])
    if meta.get("guess_supplied"):
        o["guess"] = torch.from_numpy(arr["guess"].copy()).to(dev)
    return o


@pytest.mark.parametrize("algo", ["auto", "stream", "twopass"])
@pytest.mark.parametrize("name", golden_names("gm2"))
def test_gm2_matches_reference(name, algo):
    meta, arr = golden_case(name)
    X = torch.from_numpy(arr["X"].copy()).cuda()
    o = _opts(meta, arr)
    o["algo"] = algo
    out = bz().gm2(X, o)
    res = bz().aggregators.last_result
    if meta["options"].get("maxiter", 200) == 0:
        assert out is o["guess"]                     # the guess object itself (M:184)
        return
    assert out.device.type == "cuda" and out.dtype == torch.float32
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= TOL
    assert_fixture_count(res.iters, name)
    assert torch.equal(X.cpu(), torch.from_numpy(arr["X"]))   # wList not mutated


def test_gm2_cpu_input_returns_cpu():
    meta, arr = golden_case("gm2_sgd_K50_B5")
    o = _opts(meta, arr, dev="cpu")
    out = bz().gm2(torch.from_numpy(arr["X"].copy()), o)
    assert out.device.type == "cpu"
    assert rel_l2(out.numpy(), arr["out"]) <= TOL
    assert torch.equal(o["guess"], torch.from_numpy(arr["guess"]))   # guess not mutated


def test_gm2_clamp_and_duplicates():
    meta, arr = golden_case("gm2_clamp_duplicates")
    out = bz().gm2(torch.from_numpy(arr["X"]).cuda(), _opts(meta, arr))
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= TOL
    assert_fixture_count(bz().aggregators.last_result.iters, "gm2_clamp_duplicates")


@pytest.mark.parametrize("name", golden_names("gm"))
def test_gm_host_noise_matches_reference(name):
    """AirComp gm with the reference's own draws replayed (host-injected noise)."""
    meta, arr = golden_case(name)
    o = _opts(meta, arr)
    o["noise_source"] = "host"
    torch.manual_seed(meta["rng_seed"])
    out = bz().gm(torch.from_numpy(arr["X"]).cuda(), o)
    res = bz().aggregators.last_result
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= TOL
    assert res.iters == meta["iters"]
    # the CPU generator advanced exactly as in the reference: the next draw matches
    torch.manual_seed(meta["rng_seed"])
    orc.gm(torch.from_numpy(arr["X"]), _opts(meta, arr, dev="cpu"))
    ref_next = torch.rand(4)
    torch.manual_seed(meta["rng_seed"])
    bz().gm(torch.from_numpy(arr["X"]).cuda(), o)
    assert torch.equal(torch.rand(4), ref_next)


@pytest.mark.parametrize("name", golden_names("OMA"))
def test_oma_host_noise_bit_exact(name):
    meta, arr = golden_case(name)
    X = torch.from_numpy(arr["X"].copy()).cuda()
    torch.manual_seed(meta["rng_seed"])
    bz().OMA(X, meta["noise_var"], noise_source="host")
    assert np.array_equal(X.cpu().numpy(), arr["out"])


def test_oma_philox_statistics():
    K, d, var = 64, 200_000, 1e-2
    X = torch.zeros(K, d, device="cuda")
    bz().OMA(X, var, seed=1234)
    Y = torch.zeros(K, d, device="cuda")
    bz().OMA(Y, var, seed=1234)
    assert torch.equal(X, Y)                       # counter-based: reproducible
    # per-client noise (h_r n_r + h_i n_i)/|h|^2 has variance var/|h|^2: check the
    # standardised rows are N(0,1)-like and independent across clients
    x = X.double()
    assert abs(float(x.mean())) < 5e-3
    z = x / x.std(dim=1, keepdim=True)
    assert abs(float((z ** 2).mean()) - 1.0) < 1e-2
    kurt = float((z ** 4).mean())
    assert abs(kurt - 3.0) < 0.1
    corr = float((z[0] * z[1]).mean())
    assert abs(corr) < 1e-2


@pytest.mark.parametrize("case", ["aligned", "odd_shard", "unaligned_rows", "tail"])
def test_oma_philox_matches_restatement(case):
    """Every code path of the OMA Philox kernel (float4 / scalar rows, aligned or
    odd shard offset, ragged tail) adds exactly the draws oracle/philox.py states:
    Philox4x32-10 keyed (row, column >> 2), Box-Muller in float64 there, the
    hardware log2/sqrt/sin/cos here (~1 ulp)."""
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.aggregators import Context
    from oracle.philox import oma_philox
    K, d, var, seed = 6, 4099, 1e-2, 91
    ldx, off = d, 0
    if case == "odd_shard":
        off = 2
    elif case == "unaligned_rows":
        ldx = d + 1
    elif case == "tail":
        d = ldx = 4097
    buf = torch.randn(K * ldx + 1, generator=torch.Generator().manual_seed(4)).cuda()
    Xv = buf[1:] if case == "unaligned_rows" else buf[:K * ldx]     # 4-byte misaligned
    X0 = Xv.view(K, ldx)[:, :d].cpu().numpy().copy()
    ctx = Context(buf.device.index)
    if off:
        ctx.set_shard(d + off + 5, off)
    _lib.check(ctx.lib.gm_oma_philox_f32(ctx.handle, Xv.data_ptr(), K, d, ldx, var, seed, None),
               "gm_oma_philox_f32")
    torch.cuda.synchronize()
    ctx.close()
    got = Xv.view(K, ldx)[:, :d].cpu().numpy().astype(np.float64)
    want = oma_philox(X0, var, seed, col_off=off)
    err = np.abs(got - want) / (1.0 + np.abs(want))
    assert err.max() <= 2e-6, err.max()
    assert not np.array_equal(got, X0)


@pytest.mark.parametrize("maxiter,var", [(3, 1e-2), (40, 1e-3), (25, None)])
def test_gm_philox_matches_restatement(maxiter, var):
    """The production AirComp path (Philox draws on the device) against the oracle gm
    (M:131-160, op for op) fed the same draws from oracle/philox.py: channel per
    (iteration, client), noise per (iteration, global column), denominator noise at
    index d.  Tolerance: relative L2 1e-5 (north_star), identical iteration count."""
    from oracle.philox import gm_draws
    meta, arr = golden_case("gm_var1e-2_it5")
    X = torch.from_numpy(arr["X"].copy())
    o = {"maxiter": maxiter, "tol": 1e-5, "noise_var": var, "P_max": 1}
    if meta.get("guess_supplied"):
        o["guess"] = torch.from_numpy(arr["guess"].copy())
    gpu_o = dict(o, seed=4242)
    if "guess" in o:
        gpu_o["guess"] = o["guess"].cuda()
    got = bz().gm(X.cuda(), gpu_o)
    it = bz().aggregators.last_result.iters
    draw = gm_draws(4242, X.shape[1])
    if var is None:
        draw.no_noise()
    ref, tr = orc.gm(X, o, draw=draw)
    assert it == tr.iters
    assert rel_l2(got.cpu().numpy(), ref.numpy()) <= 1e-5


def test_gm_philox_reproducible_and_close_to_ideal():
    meta, arr = golden_case("gm_var1e-2_it5")
    X = torch.from_numpy(arr["X"]).cuda()
    o = _opts(meta, arr)
    o.update(seed=77, maxiter=50)
    a = bz().gm(X, o)
    b = bz().gm(X, o)
    assert torch.equal(a, b)
    o2 = dict(o, seed=78)
    c = bz().gm(X, o2)
    assert not torch.equal(a, c)
    # noise-free AirComp must match the host-noise path's structure: with
    # noise_var=None only the channel draws differ; the aggregate stays near gm2
    ideal = bz().gm2(X, {"guess": o["guess"], "maxiter": 1000})
    assert rel_l2(a.cpu().numpy(), ideal.cpu().numpy()) < 0.05


@pytest.mark.parametrize("K,d,pad,exact", [(300, 1 << 20, 0, True), (300, 1 << 20, 4, True),
                                             (50, 1 << 22, 0, False), (1000, 65537, 0, False)])
def test_gm_rows_staged_as_panels(K, d, pad, exact):
    """Row-major AirComp gm with >= 64 passes on K*d >= 2^24 packs a panel copy once and
    streams every pass from it (api.hip gm_weiszfeld_f32).  Against the row-major passes
    (algo="stream"): bit-identical where both run the same tile (K=300, d % 4 == 0),
    relative L2 1e-5 otherwise (K=50: another tile; d odd: float1 rows); the same
    iteration count (gm runs to maxiter).  Sizes beyond the register-resident kernel;
    pad > 0: strided rows (ldx = d + pad)."""
    g = torch.Generator().manual_seed(K + d)
    X = (0.05 * torch.randn(K, d + pad, generator=g)).cuda()[:, :d]
    X[: K // 10] += 0.3
    assert X.stride(0) == d + pad
    g0 = (0.01 * torch.randn(d, generator=g)).cuda()
    o = {"maxiter": 64, "tol": 1e-5, "noise_var": 1e-2, "P_max": 1, "seed": 99, "guess": g0}
    a = bz().gm(X, o)
    ra = bz().aggregators.last_result
    b = bz().gm(X, dict(o, algo="stream"))
    rb = bz().aggregators.last_result
    assert (ra.iters, ra.algo) == (rb.iters, rb.algo) == (64, "stream")
    if exact:
        assert torch.equal(a, b)
    else:
        assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-5


SHAPE_K = [1, 2, 16, 17, 33, 64, 65, 129, 257, 513, 1000, 1025, 2049]
SHAPE_D = [1, 6, 4099]


def _sgd_like(K, d, seed):
    g = torch.Generator().manual_seed(seed)
    p = 0.07 * torch.randn(d, generator=g)
    X = p + 5e-4 * torch.randn(K, d, generator=g)
    B = K // 5
    if B:
        X[K - B:] += 5e-3 * torch.randn(B, d, generator=g) + 2e-3
    return X, p


@pytest.mark.parametrize("K", SHAPE_K)
@pytest.mark.parametrize("d", SHAPE_D)
def test_gm2_shapes_vs_oracle(K, d):
    X, p = _sgd_like(K, d, K * 7919 + d)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": p.clone()}
    want, tr = orc.gm2(X.clone(), dict(opts))
    got = bz().gm2(X.cuda(), dict(opts, guess=p.cuda()))
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= TOL
    assert abs(bz().aggregators.last_result.iters - tr.iters) <= ITER_SLACK


def test_gm2_strided_rows():
    meta, arr = golden_case("gm2_sgd_K50_B10")
    K, d = arr["X"].shape
    big = torch.zeros(K, d + 6)
    big[:, :d] = torch.from_numpy(arr["X"])
    view = big.cuda()[:, :d]                     # ldx = d + 6, not contiguous
    out = bz().gm2(view, _opts(meta, arr))
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= TOL


def test_gm2_nan_runs_to_maxiter():
    X = torch.randn(8, 100, generator=torch.Generator().manual_seed(8))
    X[3, 7] = float("nan")
    out = bz().gm2(X.cuda(), {"maxiter": 13})
    assert bz().aggregators.last_result.iters == 13
    assert torch.isnan(out).all()


def test_gm2_default_options_mean_guess():
    meta, arr = golden_case("gm2_defaults")
    out = bz().gm2(torch.from_numpy(arr["X"]).cuda())
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= TOL
    assert_fixture_count(bz().aggregators.last_result.iters, "gm2_defaults")


def test_gm2_translation_and_permutation_invariance():
    g = torch.Generator().manual_seed(5)
    X = (0.05 * torch.randn(300, 50_000, generator=g)).cuda()
    X[240:] += 0.25
    base = bz().gm2(X, {"maxiter": 100, "tol": 1e-6})
    perm = torch.randperm(300, generator=g).cuda()
    moved = bz().gm2(X[perm], {"maxiter": 100, "tol": 1e-6})
    assert rel_l2(moved.cpu().numpy(), base.cpu().numpy()) < 1e-5
    shift = bz().gm2(X + 1.0, {"maxiter": 100, "tol": 1e-6})
    assert rel_l2((shift - 1.0).cpu().numpy(), base.cpu().numpy()) < 1e-4


def test_gm2_large_fixed_point_property():
    """Full-size-style check: at the returned g, sum_k (x_k - g)/d_k ~ 0 (Weiszfeld optimality)."""
    m = bz()
    K, d = 1000, 2_000_000
    X = torch.empty(K, d, device="cuda")
    ctx = m.context()
    m._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, 200, 0.0, 0.05,
                                             0.25, 0.5, 20211, torch.cuda.current_stream().cuda_stream),
                 "fill")
    g0 = torch.empty(d, device="cuda")
    m._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, 20212,
                                            torch.cuda.current_stream().cuda_stream), "fill")
    g = m.gm2(X, {"maxiter": 1000, "tol": 1e-5, "guess": g0})
    res = m.aggregators.last_result
    # the count: against the exact (fp64, on the device) iteration's window, +-1
    window = orc.gm2_count_window(X, g0, 1000, 1e-5)
    assert res.converged and window.determined and window.width <= 1, (res, window)
    assert_iter_count(res.iters, window.late, window)
    dist = torch.stack([torch.linalg.vector_norm((X[k0:k0 + 100].double() - g.double()), dim=1)
                        for k0 in range(0, K, 100)]).flatten().clamp_min(1e-4)
    w = 1.0 / dist
    grad = torch.zeros(d, dtype=torch.float64, device="cuda")
    for k0 in range(0, K, 100):
        grad += (w[k0:k0 + 100, None] * (X[k0:k0 + 100].double() - g.double())).sum(0)
    # grad / sum(w) is the next Weiszfeld step g' - g: at convergence its norm is
    # of the order of the tol-test movement
    assert float(grad.norm() / w.sum()) < 1e-4


# --- Gram-space variant (north_star's second design) ---------------------------

@pytest.mark.parametrize("algo", ["gram", "gram_f32"])
@pytest.mark.parametrize("name", golden_names("gm2"))
def test_gram_matches_reference(name, algo):
    meta, arr = golden_case(name)
    K, d = arr["X"].shape
    o = _opts(meta, arr)
    o["algo"] = algo
    X = torch.from_numpy(arr["X"].copy()).cuda()
    if meta["options"].get("maxiter", 200) == 0:
        assert bz().gm2(X, o) is o["guess"]
        return
    if d % 4 or K > 256:
        with pytest.raises(bz()._lib.GmError):
            bz().gm2(X, o)
        return
    out = bz().gm2(X, o)
    res = bz().aggregators.last_result
    assert res.algo == algo
    assert rel_l2(out.cpu().numpy(), arr["out"]) <= TOL
    assert_fixture_count(res.iters, name)


GRAM_K = [1, 8, 32, 33, 64, 100, 128, 200, 256]
GRAM_D = [4, 4096, 100_000]


@pytest.mark.parametrize("algo", ["gram", "gram_f32"])
@pytest.mark.parametrize("K", GRAM_K)
@pytest.mark.parametrize("d", GRAM_D)
def test_gram_shapes_vs_oracle(K, d, algo):
    X, p = _sgd_like(K, d, K * 31 + d)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": p.clone()}
    want, tr = orc.gm2(X.clone(), dict(opts))
    got = bz().gm2(X.cuda(), dict(opts, guess=p.cuda(), algo=algo))
    assert bz().aggregators.last_result.algo == algo
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= TOL
    assert abs(bz().aggregators.last_result.iters - tr.iters) <= ITER_SLACK


def test_gram_matches_stream_at_c4_scale():
    """K=256 x d=4M synthetic (C4 recipe): Gram and streaming agree."""
    m = bz()
    K, d = 256, 4_000_000
    X = torch.empty(K, d, device="cuda")
    ctx = m.context()
    s = torch.cuda.current_stream().cuda_stream
    m._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, 51, 0.0, 0.05,
                                             0.25, 0.5, 20211, s), "fill")
    g0 = torch.empty(d, device="cuda")
    m._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, 20212, s),
                 "fill")
    a = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "stream"})
    na = m.aggregators.last_result.iters
    b = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "gram"})
    nb = m.aggregators.last_result.iters
    assert abs(na - nb) <= 1
    assert rel_l2(b.cpu().numpy(), a.cpu().numpy()) <= TOL


def _c4_like(K, d, seed=20211):
    m = bz()
    X = torch.empty(K, d, device="cuda")
    ctx = m.context()
    s = torch.cuda.current_stream().cuda_stream
    m._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, K // 5, 0.0, 0.05,
                                             0.25, 0.5, seed, s), "fill")
    g0 = torch.empty(d, device="cuda")
    m._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, seed + 1, s),
                 "fill")
    return X, g0


def test_gram_split_vs_f32_and_auto_choice():
    """The scaled-f16 split Gram (algo="gram") agrees with the exact f32-MFMA Gram; AUTO keeps it
    (guard passes)."""
    m = bz()
    X, g0 = _c4_like(256, 1 << 20)
    a = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "gram_f32"})
    na = m.aggregators.last_result.iters
    b = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "gram"})
    nb = m.aggregators.last_result.iters
    c = m.gm2(X, {"maxiter": 1000, "guess": g0})
    assert m.aggregators.last_result.algo == "gram"
    assert na == nb and abs(m.aggregators.last_result.iters - nb) == 0
    assert rel_l2(b.cpu().numpy(), a.cpu().numpy()) <= 1e-6
    assert rel_l2(c.cpu().numpy(), b.cpu().numpy()) <= 1e-6   # closing-pass tiles differ


GUARD_CASES = ["far_offset", "tight_cluster", "g_error"]


def _guard_data(case):
    g = torch.Generator().manual_seed(11)
    K, d = 64, 1 << 18
    if case == "far_offset":
        X = 3.0 + 0.05 * torch.randn(K, d, generator=g)
    elif case == "tight_cluster":
        X = 1.0 + 1e-3 * torch.randn(K, d, generator=g)
        X[50:] += 0.05
    else:            # ||g|| small enough for the floor test; D_k ~ 1e-7 G_kk
        X = 0.05 + 1e-5 * torch.randn(K, d, generator=g)
    return X, torch.zeros(d)


@pytest.mark.parametrize("shift", [0.0, 0.07])
def test_gram_c4_recipe_vs_oracle(shift):
    """north_star's second design on the C4 recipe (K = 256, d = 2^20), AUTO, against the
    oracle gm2.  shift = 0: ||g|| ~ 6.8, the fp32 movement floor (2^-23 ||g||) far below
    tol/3: guard 'accepted', iterations +-1.  shift = 0.07 (every element and the guess;
    the algorithm is translation-invariant, the rounding is not): ||g|| ~ 72, the floor
    8.6e-6 between tol/3 and tol — the whole C4 job's regime (||g|| = 74 at d = 125M):
    guard 'accepted_floor'; the Gram's exact-arithmetic count must equal the fp32 oracle's
    count +-1 AND the streaming path's count +-1 (measured: 5, 5, 5), and lie in the
    count window (determined there: [4, 5]); the aggregate to 1e-5 of both the oracle and
    the streaming path."""
    m = bz()
    X, g0 = _c4_like(256, 1 << 20, seed=4040)
    X += shift
    g0 += shift
    got = m.gm2(X, {"maxiter": 1000, "guess": g0})
    res = m.aggregators.last_result
    assert res.algo == "gram"
    assert res.guard == ("accepted" if shift == 0.0 else "accepted_floor"), res
    Xc, gc = X.cpu(), g0.cpu()
    want, tr = orc.gm2(Xc, {"maxiter": 1000, "tol": 1e-5, "guess": gc.clone()})
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= TOL
    assert abs(res.iters - tr.iters) <= ITER_SLACK, (res, tr)
    s = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "stream"})
    rs = m.aggregators.last_result
    assert rs.algo == "stream" and abs(res.iters - rs.iters) <= ITER_SLACK, (res, rs)
    assert rel_l2(got.cpu().numpy(), s.cpu().numpy()) <= TOL
    if shift:
        window = orc.gm2_count_window(Xc, gc, 1000, 1e-5)
        assert window.determined, window          # the guard and the window share one floor
        assert_iter_count(res.iters, tr.iters, window)


@pytest.mark.parametrize("case", GUARD_CASES)
def test_gram_guard_falls_back_to_streaming(case):
    """Data where the Gram may not reproduce the reference: the reference's fp32
    movement floor ~2^-24 ||g|| exceeds tol/3 (AUTO must run the streaming path),
    or D_k ~ 1e-7 G_kk (the a-posteriori check decides; either way the result
    must match the oracle)."""
    m = bz()
    X, p = _guard_data(case)
    opts = {"maxiter": 30, "tol": 1e-5, "guess": p}
    want, tr = orc.gm2(X.clone(), dict(opts))
    got = m.gm2(X.cuda(), dict(opts, guess=p.cuda()))
    res = m.aggregators.last_result
    if case != "g_error":            # the floor test alone decides these
        assert res.algo == "stream"
    # whichever path AUTO kept, it reproduces the reference
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= TOL
    window = orc.gm2_count_window(X, p, 30, 1e-5)
    if case == "g_error":
        assert_iter_count(res.iters, tr.iters, window)
    else:
        # far_offset / tight_cluster put tol far below the fp32 movement floor by design
        # (||g|| 1536 / 517: floor 18x / 6x tol): maxiter, as the reference (30), or an exact
        # fp32 fixed point (measured: rows streaming stops at 9 with movement 0 on
        # far_offset, every other path runs 30)
        assert tr.iters == 30
        assert_floor_count(res, 30, window)


def test_gram_f16_split_matches_bf16_split(monkeypatch):
    """The scaled f16 split (3 MFMA products, default) and the bf16 split (4
    products) give the same aggregate and iterations on the C4 recipe."""
    m = bz()
    X, g0 = _c4_like(256, 1 << 20, seed=777)
    a = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "gram"})
    ra = m.aggregators.last_result
    monkeypatch.setenv("GMAGG_GRAM_KIND", "bf16")
    b = m.gm2(X, {"maxiter": 1000, "guess": g0, "algo": "gram"})
    rb = m.aggregators.last_result
    assert (ra.gram_kind, rb.gram_kind) == ("f16_split", "bf16_split")
    assert ra.guard == rb.guard == "accepted" and ra.iters == rb.iters
    assert rel_l2(a.cpu().numpy(), b.cpu().numpy()) <= 1e-6


def _spike_data(spike):
    g = torch.Generator().manual_seed(5)
    K, d = 64, 1 << 18
    X = 0.05 * torch.randn(K, d, generator=g)
    X[K - 12:] += 0.25
    X[5, 200_000] = spike                     # well past the first stages of its block
    return X, torch.zeros(d)


@pytest.mark.parametrize("spike", [1e6, float("inf")])
def test_gram_f16_range_overflow_falls_back(spike):
    """An element far beyond the f16 headroom of its row's scale (set from the
    block's first stages) makes the f16 Gram non-finite: the call reruns the bf16
    split (or, for a non-finite input, ends on the streaming path) and still
    matches the reference."""
    m = bz()
    X, p = _spike_data(spike)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": p}
    want, tr = orc.gm2(X.clone(), dict(opts))
    got = m.gm2(X.cuda(), dict(opts, guess=p.cuda(), algo="gram"))
    res = m.aggregators.last_result
    if spike == float("inf"):
        assert res.algo == "stream" and res.guard == "rejected"
        assert torch.equal(torch.isnan(got.cpu()), torch.isnan(want))
        return
    assert res.algo == "gram" and res.gram_kind == "bf16_split"
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= TOL
    assert abs(res.iters - tr.iters) <= ITER_SLACK


@pytest.mark.parametrize("K,d,layout,algo", [
    (1000, 4096, "rows", "stream"),       # fused into the INIT pass (float4 rows)
    (1000, 4100, "panels", "auto"),       # fused, panels (partial last float4 group of panels)
    (300, 2051, "rows", "stream"),        # float1 rows: the standalone OMA first
    (50, 7850, "rows", "auto"),           # register-resident path: standalone OMA first
    (50, 7850, "panels", "auto"),         # batched resident kernel, P = 1: fused in registers
    (12, 30_001, "panels", "resident"),
    (256, 1 << 18, "rows", "auto"),       # guarded Gram: standalone OMA first
    (200, (1 << 18) + 64, "panels", "auto"),
])
def test_pre_oma_equals_oma_then_gm2(K, d, layout, algo):
    """gm2 with pre_oma_var (the reference's OMA(weight_f, var) before the aggregator,
    M:351-352) == OMA then gm2: the same noisy X, bit for bit, and the same aggregate."""
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K + d)
    X = 0.05 * torch.randn(K, d, generator=g)
    X[K - K // 5:] += 0.25
    g0 = (0.01 * torch.randn(d, generator=g)).cuda()
    X = X.cuda()

    def fresh():
        return bz.ClientPanels.from_rows(X) if layout == "panels" else X.clone()

    opts = {"maxiter": 30, "tol": 1e-5, "guess": g0, "algo": algo}
    A = fresh()
    bz.OMA(A, 1e-2, seed=77)
    a = bz.gm2(A, dict(opts))
    ra = bz.aggregators.last_result
    B = fresh()
    b = bz.gm2(B, dict(opts, pre_oma_var=1e-2, pre_oma_seed=77))
    rb = bz.aggregators.last_result
    da = A.data if layout == "panels" else A
    db = B.data if layout == "panels" else B
    assert torch.equal(da, db)
    assert torch.equal(a, b)
    assert (ra.iters, ra.algo) == (rb.iters, rb.algo)


@pytest.mark.parametrize("layout,d", [("rows", 10000), ("panels", 10000), ("rows", 1001),
                                      ("panels", 1001)])
def test_batched_pre_oma_equals_oma_then_gm2(layout, d):
    """(rows at d % 4 != 0 take the float1 tile: the standalone batched OMA runs first)"""
    from byzantine_aircomp_amd.batched import ProblemPanels, gm2_batched, oma_batched
    P, K = 6, 50
    g = torch.Generator().manual_seed(3)
    X = (0.05 * torch.randn(P, K, d, generator=g)).cuda()
    g0 = (0.01 * torch.randn(P, d, generator=g)).cuda()

    def fresh():
        return ProblemPanels.from_rows(X) if layout == "panels" else X.clone()

    opts = {"maxiter": 30, "tol": 1e-5, "guess": g0}
    A = fresh()
    oma_batched(A, 1e-2, seed=123)
    a, ra = gm2_batched(A, dict(opts))
    B = fresh()
    b, rb = gm2_batched(B, dict(opts, pre_oma_var=1e-2, pre_oma_seed=123))
    da = A.data if layout == "panels" else A
    db = B.data if layout == "panels" else B
    assert torch.equal(da, db)
    assert torch.equal(a, b)
    assert [r.iters for r in ra] == [r.iters for r in rb]


def test_pre_oma_strided_view_is_noised_in_place():
    """A strided [K, d] view (ldx = d + 3, unaligned for float4) is packed into a copy for
    the kernels; the fused pre-noise must still land in the caller's tensor, as OMA()
    does (M:351-352 mutates weight_f in place).  Single, batched and sharded calls."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.batched import gm2_batched, oma_batched
    K, d = 300, 4096
    g = torch.Generator().manual_seed(12)
    base = (0.05 * torch.randn(K, d + 3, generator=g)).cuda()
    g0 = (0.01 * torch.randn(d, generator=g)).cuda()
    opts = {"maxiter": 30, "tol": 1e-5, "guess": g0}
    ref = base[:, :d].clone()
    bz.OMA(ref, 1e-2, seed=5)
    want = bz.gm2(ref, dict(opts))
    big = base.clone()
    view = big[:, :d]
    assert not view.is_contiguous()
    got = bz.gm2(view, dict(opts, pre_oma_var=1e-2, pre_oma_seed=5))
    assert torch.equal(view, ref)
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6
    # batched: a [P, K, d] view with padded rows
    P = 3
    bb = (0.05 * torch.randn(P, 50, d + 4, generator=g)).cuda()
    gb = (0.01 * torch.randn(P, d, generator=g)).cuda()
    vref = bb[:, :, :d].clone()
    oma_batched(vref, 1e-2, seed=9)
    vb = bb[:, :, :d]
    vb = vb.transpose(0, 1).contiguous().transpose(0, 1)     # non-standard problem stride
    gm2_batched(vb, {"maxiter": 30, "tol": 1e-5, "guess": gb, "pre_oma_var": 1e-2,
                     "pre_oma_seed": 9})
    assert torch.equal(vb, vref)
    # the default guess (the mean of the NOISY rows): the separate OMA runs first, on the
    # packed copy, and must land in the caller's view as well
    vc = bb[:, :, :d].transpose(0, 1).contiguous().transpose(0, 1)
    gm2_batched(vc, {"maxiter": 30, "tol": 1e-5, "pre_oma_var": 1e-2, "pre_oma_seed": 9})
    assert torch.equal(vc, vref)


def test_pre_oma_host_draws_keep_reference_sequence():
    """With noise_source='host' the pre-noise replays the reference's torch.normal draws
    (M:389-392); the call must not consume any other draw from the CPU generator first,
    so OMA + gm2 here equals the oracle's OMA then gm2 from the same generator state."""
    import byzantine_aircomp_amd as bz
    K, d = 20, 1000
    g = torch.Generator().manual_seed(3)
    X = 0.05 * torch.randn(K, d, generator=g)
    p = 0.01 * torch.randn(d, generator=g)
    torch.manual_seed(4321)
    Xr = X.clone()
    orc.oma_(Xr, 1e-2)
    want, _ = orc.gm2(Xr, {"maxiter": 100, "tol": 1e-5, "guess": p.clone()})
    after_ref = torch.randint(0, 2 ** 30, (1,)).item()
    torch.manual_seed(4321)
    Xg = X.clone().cuda()
    got = bz.gm2(Xg, {"maxiter": 100, "tol": 1e-5, "guess": p.cuda(), "pre_oma_var": 1e-2,
                      "noise_source": "host"})
    after_gpu = torch.randint(0, 2 ** 30, (1,)).item()
    assert after_ref == after_gpu              # the same number of CPU-generator draws
    assert torch.equal(Xg.cpu(), Xr)
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= TOL


def iteration_cases():
    """The +-1 inputs above, on the CPU (tests/test_iteration_wellposed.py); the
    device-filled C4-recipe inputs through oracle/philox_fill.c.  Not here: the
    Gram-vs-streaming equality at K = 256 x d = 4M (test_gram_matches_stream_at_c4_scale):
    16 GB of fp64 for the exact iteration; its ||g|| ~ 13 puts delta at 3.1e-6."""
    from conftest import golden_case, golden_names
    cases = []
    for name in golden_names("gm2"):
        def t(name=name):
            meta, arr = golden_case(name)
            o = meta["options"]
            guess = torch.from_numpy(arr["guess"].copy()) if meta.get("guess_supplied") else None
            # (assert_fixture_count: the window, or the fixture's stated slack)
            return [(torch.from_numpy(arr["X"].copy()), guess, o.get("maxiter", 200),
                     o.get("tol", 1e-5), "undetermined" if name in FIXTURE_SLACK else "windowed")]
        cases.append((f"golden_{name}", t))
    for K in SHAPE_K:
        def t(K=K):
            out = []
            for d in SHAPE_D:
                X, p = _sgd_like(K, d, K * 7919 + d)
                out.append((X, p, 1000, 1e-5))
            return out
        cases.append((f"shapes_K{K}", t))
    for K in GRAM_K:
        def t(K=K):
            out = []
            for d in GRAM_D:
                X, p = _sgd_like(K, d, K * 31 + d)
                out.append((X, p, 1000, 1e-5))
            return out
        cases.append((f"gram_K{K}", t))
    for case in GUARD_CASES:
        def t(case=case):
            X, p = _guard_data(case)
            return [(X, p, 30, 1e-5, "windowed" if case == "g_error" else "undetermined")]
        cases.append((f"guard_{case}", t))
    cases.append(("spike", lambda: [(*_spike_data(1e6), 1000, 1e-5)]))
    from oracle.philox import fill_clients, fill_normal

    def c4_like(K, d, seed=20211, shift=0.0, flag=()):
        X = torch.from_numpy(fill_clients(K, d, K // 5, 0.0, 0.05, 0.25, 0.5, seed)) + shift
        g0 = torch.from_numpy(fill_normal(d, 0.0, 0.01, seed + 1)) + shift
        return [(X, g0, 1000, 1e-5, *flag)]
    # (_c4_like on the device: gram_split_vs_f32 seed 20211, f16_vs_bf16 seed 777, the C4
    # recipe vs the oracle seed 4040, shifted by 0.07 into the floor band: windowed)
    cases.append(("c4like_256x2^20_s20211", lambda: c4_like(256, 1 << 20)))
    cases.append(("c4like_256x2^20_s777", lambda: c4_like(256, 1 << 20, seed=777)))
    cases.append(("c4like_256x2^20_s4040", lambda: c4_like(256, 1 << 20, seed=4040)))
    cases.append(("c4like_256x2^20_s4040_shift", lambda: c4_like(256, 1 << 20, seed=4040,
                                                                 shift=0.07, flag=("windowed",))))
    return cases


@pytest.mark.parametrize("agg", ["gm2", "gm"])
def test_resident_xcd_local_exchange_matches_agent_scope(agg, monkeypatch):
    """C2's single-problem resident kernel: its 31 blocks on one XCD with the granules kept
    in that XCD's L2 (GMAGG_RES_XCD=2, the default; resident.hip put_value) against the
    blocks dealt over every XCD with agent-scope granule stores (GMAGG_RES_XCD=0).  The
    exchange carries the same values in the same order, only where they are cached
    differs, so the results are bit-identical."""
    X, p = _sgd_like(50, 7850, 2718)
    X, p = X.cuda(), p.cuda()
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": p}
    if agg == "gm":
        opts.update(maxiter=200, noise_var=1e-2, seed=5)
    f = getattr(bz(), agg)
    outs = {}
    for mode in ("2", "0"):
        monkeypatch.setenv("GMAGG_RES_XCD", mode)
        outs[mode] = (f(X.clone(), dict(opts)).cpu(), bz().aggregators.last_result)
    (a, ra), (b, rb) = outs["2"], outs["0"]
    assert ra.algo == "resident" and rb.algo == "resident"
    assert ra.iters == rb.iters
    assert torch.equal(a, b)
