"""d-sharded aggregation through libgmagg's real host loop, on ONE GPU.

P "virtual ranks" run in P threads, each with its own context holding a column
shard; their all-reduce callback sums the (K+2)-vectors across threads.  The
sharded result must equal the unsharded one: for gm2 to fp32 reduction order,
and for AirComp gm with Philox noise too (draws are keyed by global index, so
shards regenerate the same channel and noise without communicating).  The
native RCCL path is exercised with a single-rank communicator (one GPU here).
"""
import ctypes as C
import threading

import pytest
import torch

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _problem_cpu(K, d, B, seed):
    g = torch.Generator().manual_seed(seed)
    p = 0.07 * torch.randn(d, generator=g)
    X = p + 5e-4 * torch.randn(K, d, generator=g)
    X[K - B:] = p + 5e-3 * torch.randn(B, d, generator=g) + 2e-3
    return X, p


def _problem(K, d, B, seed):
    X, p = _problem_cpu(K, d, B, seed)
    return X.cuda(), p.cuda()


def _sharded(X, p, P, opts, aircomp, check_every=0, algo=0, panels=False):
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.aggregators import Context
    from byzantine_aircomp_amd.sharded import _wrap, shard_range

    K, d = X.shape
    dev = X.device
    barrier = threading.Barrier(P, timeout=60)   # a rank-dependent collective count fails here
    bufs = [None] * P
    out = [None] * P
    errs = []

    def run(r):
        try:
            lo, hi = shard_range(d, P, r)
            ctx = Context(dev.index)
            ctx.set_shard(d, lo)

            def allreduce(ptr, count, stream):
                torch.cuda.synchronize(dev)
                t = _wrap(ptr, count, dev)
                bufs[r] = t.clone()
                barrier.wait()
                total = torch.stack(bufs).sum(0)
                barrier.wait()
                t.copy_(total)
                torch.cuda.synchronize(dev)
            ctx.set_allreduce(allreduce)
            Xs = X[:, lo:hi].contiguous()
            ptr, ldx = Xs.data_ptr(), hi - lo
            if panels:
                from byzantine_aircomp_amd import ClientPanels
                Xs = ClientPanels.from_rows(Xs)
                ptr, ldx = Xs.data.data_ptr(), Xs.panel_stride
            g0 = p[lo:hi].contiguous()
            res = torch.empty(hi - lo, device=dev)
            o = _lib.GmOpts()
            o.maxiter, o.tol, o.eps = opts["maxiter"], opts["tol"], 1e-4
            o.mode = _lib.GM_MODE_AIRCOMP if aircomp else _lib.GM_MODE_IDEAL
            o.check_every, o.algo = check_every, algo
            o.layout = _lib.GM_LAYOUT_PANELS if panels else _lib.GM_LAYOUT_ROWS
            if aircomp:
                o.has_noise, o.noise_var, o.P_max, o.seed = 1, opts["noise_var"], 1.0, opts["seed"]
            rr = _lib.GmResult()
            _lib.check(ctx.lib.gm_weiszfeld_f32(ctx.handle, ptr, K, hi - lo, ldx,
                                                g0.data_ptr(), res.data_ptr(), C.byref(o),
                                                C.byref(rr), None), "sharded gm")
            torch.cuda.synchronize(dev)
            out[r] = (lo, hi, res, rr.iters, rr.algo_used, rr.guard)
        except Exception as e:  # noqa: BLE001
            errs.append(e)
            barrier.abort()

    th = [threading.Thread(target=run, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=120)
    assert not errs, errs
    full = torch.empty(d, device=dev)
    iters = {o_[3] for o_ in out}
    _sharded.algos = {o_[4] for o_ in out}
    _sharded.guards = {o_[5] for o_ in out}
    for lo, hi, res, _, _, _ in out:
        full[lo:hi] = res
    return full, iters


@pytest.mark.parametrize("P", [2, 3, 4])
def test_sharded_gm2_equals_unsharded(P):
    import byzantine_aircomp_amd as bz
    X, p = _problem(200, 50_000, 40, seed=P)
    opts = {"maxiter": 1000, "tol": 1e-5}
    want = bz.gm2(X, dict(opts, guess=p))
    n = bz.aggregators.last_result.iters
    got, iters = _sharded(X, p, P, opts, aircomp=False)
    assert iters == {n} or max(abs(i - n) for i in iters) <= 1
    assert len(iters) == 1                          # every shard took the same decisions
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


def test_sharded_gm_philox_equals_unsharded():
    import byzantine_aircomp_amd as bz
    X, p = _problem(50, 7850 * 4, 10, seed=9)
    opts = {"maxiter": 40, "tol": 1e-5, "noise_var": 1e-2, "seed": 4242}
    want = bz.gm(X, dict(opts, guess=p))
    got, iters = _sharded(X, p, 2, opts, aircomp=True)
    assert iters == {40}
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-5


def test_rccl_single_rank_path():
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.aggregators import Context
    X, p = _problem(64, 10_000, 12, seed=3)
    want = bz.gm2(X, {"maxiter": 1000, "guess": p})
    ctx = Context(X.device.index)
    buf = C.create_string_buffer(128)
    _lib.check(ctx.lib.gm_rccl_get_unique_id(buf), "uid")
    ctx.init_rccl(buf.raw, 1, 0)
    ctx.set_shard(10_000, 0)
    out = torch.empty(10_000, device="cuda")
    o = _lib.GmOpts()
    o.maxiter, o.tol, o.eps = 1000, 1e-5, 1e-4
    rr = _lib.GmResult()
    _lib.check(ctx.lib.gm_weiszfeld_f32(ctx.handle, X.data_ptr(), 64, 10_000, 10_000, p.data_ptr(),
                                        out.data_ptr(), C.byref(o), C.byref(rr), None), "rccl gm2")
    torch.cuda.synchronize()
    assert rel_l2(out.cpu().numpy(), want.cpu().numpy()) <= 1e-7


@pytest.mark.parametrize("P", [2, 3])
def test_sharded_lagged_poll_equals_unsharded(P):
    """check_every = 1: every rank reads iteration t-1's state while t is queued
    (the large-problem host loop); all ranks must stop together."""
    import byzantine_aircomp_amd as bz
    X, p = _problem(200, 50_000, 40, seed=10 + P)
    opts = {"maxiter": 1000, "tol": 1e-5}
    want = bz.gm2(X, dict(opts, guess=p, check_every=1))
    n = bz.aggregators.last_result.iters
    got, iters = _sharded(X, p, P, opts, aircomp=False, check_every=1)
    assert len(iters) == 1 and abs(iters.pop() - n) <= 1
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


def _gram_data():
    K, d = 64, 2 * (1 << 18) + 4096
    g = torch.Generator().manual_seed(21)         # C4 recipe: the guard keeps the Gram result
    X = 0.05 * torch.randn(K, d, generator=g)
    X[K - 12:] = 0.25 + 0.5 * torch.randn(12, d, generator=g)
    return X, 0.01 * torch.randn(d, generator=g)


@pytest.mark.parametrize("algo", [0, 3])          # AUTO (guarded Gram) and explicit split Gram
def test_sharded_gram_equals_unsharded(algo):
    """d-sharded Gram: one all-reduce of G (and of the closing pass's sums for the
    guard); every rank takes the same guard decision."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    P = 2
    X, p = _gram_data()
    X, p = X.cuda(), p.cuda()
    opts = {"maxiter": 1000, "tol": 1e-5}
    want = bz.gm2(X, dict(opts, guess=p, algo="stream"))
    n = bz.aggregators.last_result.iters
    got, iters = _sharded(X, p, P, opts, aircomp=False, algo=algo)
    assert len(iters) == 1 and abs(iters.pop() - n) <= 1
    assert len(_sharded.algos) == 1
    info = (_sharded.algos, _sharded.guards, bz.aggregators.last_result)
    if algo == 3:
        bz.gm2(X, dict(opts, guess=p, algo="gram"))
        info = info + (bz.aggregators.last_result,)
        assert _sharded.algos == {_lib.GM_ALGO_GRAM}, info
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("P", [2, 3])
@pytest.mark.parametrize("check_every", [0, 1])
def test_sharded_panels_equal_sharded_rows(P, check_every):
    """Each rank's shard in the panel layout against the row-major shard (d_local % 4 == 0):
    the same chunks per block, the same iteration count; at K = 1000 the row-major gm2
    passes run the 32-wave rows kernel (rows_pass.hip), which sums a column's rows in
    another order, so the results agree to rounding (bit for bit before round 6)."""
    X, p = _problem(1000, 40_960, 200, seed=20 + P)
    opts = {"maxiter": 1000, "tol": 1e-5}
    rows, it_r = _sharded(X, p, P, opts, aircomp=False, check_every=check_every, algo=1)
    pan, it_p = _sharded(X, p, P, opts, aircomp=False, check_every=check_every, algo=1,
                         panels=True)
    assert it_r == it_p and len(it_p) == 1
    assert rel_l2(rows.cpu().numpy(), pan.cpu().numpy()) <= 1e-6


def test_sharded_gm_panels_philox():
    X, p = _problem(300, 8192, 60, seed=31)
    opts = {"maxiter": 30, "tol": 1e-5, "noise_var": 1e-2, "seed": 77}
    rows, _ = _sharded(X, p, 2, opts, aircomp=True, algo=1)
    pan, it = _sharded(X, p, 2, opts, aircomp=True, algo=1, panels=True)
    assert it == {30}
    assert rel_l2(pan.cpu().numpy(), rows.cpu().numpy()) <= 1e-6


@pytest.mark.parametrize("cuts", [(0, 4096, 8192, 10_001), (0, 4097, 6000, 10_001)])
def test_oma_philox_shard_invariant(cuts):
    """OMA's Philox draws are keyed by (row, global column pair): a shard at any
    column offset (even or odd, float4 or scalar path) regenerates exactly the
    noise the unsharded call adds to its columns."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.aggregators import Context
    K, d = 7, 10_001
    X = torch.randn(K, d, generator=torch.Generator().manual_seed(3)).cuda()
    full = X.clone()
    bz.OMA(full, 1e-2, seed=5)
    assert not torch.equal(full, X)
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        ctx = Context(X.device.index)
        ctx.set_shard(d, lo)
        part = X[:, lo:hi].contiguous()
        from byzantine_aircomp_amd import _lib
        _lib.check(ctx.lib.gm_oma_philox_f32(ctx.handle, part.data_ptr(), K, hi - lo, hi - lo,
                                             1e-2, 5, None), "oma shard")
        torch.cuda.synchronize()
        assert torch.equal(part, full[:, lo:hi]), (lo, hi)
        ctx.close()


RAGGED = [
    # 1000 x 50002 over 3: shards 16896 / 16896 / 16210 columns (last ragged, d % 4 = 2);
    # K * d_local straddles the 2^24 poll threshold, K * d_total does not
    (1000, 50_002, 3, 0, {1}),
    (1000, 50_002, 3, 1, {1}),
    # d_total >= 2^18 with every shard below it: AUTO takes Gram on d_total (all ranks)
    (200, (1 << 18) + 1024, 3, 0, {3}),
    # d_total % 4 == 2: no Gram anywhere, although the first shards are float4-aligned
    (200, (1 << 18) + 1026, 3, 0, {1}),
]


def _ragged_data(K, d):
    g = torch.Generator().manual_seed(d % 1000)    # the C3/C4 recipe
    B = K // 5
    X = 0.05 * torch.randn(K, d, generator=g)
    X[K - B:] = 0.25 + 0.5 * torch.randn(B, d, generator=g)
    return X, 0.01 * torch.randn(d, generator=g)


@pytest.mark.parametrize("K,d,P,algo,want_algo", RAGGED)
def test_sharded_ragged_last_shard_same_decisions(K, d, P, algo, want_algo):
    """Every rank must issue the same sequence of all-reduces: the
    Gram/streaming choice and the poll interval come from K, d_total and the
    options, never from the local slice."""
    import byzantine_aircomp_amd as bz
    X, p = _ragged_data(K, d)
    X, p = X.cuda(), p.cuda()
    opts = {"maxiter": 1000, "tol": 1e-5}
    want = bz.gm2(X, dict(opts, guess=p, algo="stream"))
    n = bz.aggregators.last_result.iters
    got, iters = _sharded(X, p, P, opts, aircomp=False, algo=algo)
    assert len(iters) == 1 and abs(iters.pop() - n) <= 1
    assert _sharded.algos == want_algo
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-5


def iteration_cases():
    """The +-1 inputs above, on the CPU (tests/test_iteration_wellposed.py)."""
    cases = []
    for seed in (2, 3, 4, 12, 13):          # test_sharded_gm2_equals_unsharded, lagged poll
        cases.append((f"sgd_seed{seed}",
                      lambda seed=seed: [(*_problem_cpu(200, 50_000, 40, seed), 1000, 1e-5)]))
    cases.append(("gram", lambda: [(*_gram_data(), 1000, 1e-5)]))
    for K, d in sorted({(K, d) for K, d, *_ in RAGGED}):
        cases.append((f"ragged_{K}x{d}", lambda K=K, d=d: [(*_ragged_data(K, d), 1000, 1e-5)]))
    return cases
