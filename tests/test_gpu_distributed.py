"""The multi-GPU API (sharded.ShardedGM) executed through real torch.distributed
process groups on the test box's GPU.

One process per GPU is the production shape (bench.py / INTEGRATION.md); a
one-GPU box can host a world of size 1, so these tests start an in-process
group (tcp://127.0.0.1, gloo and nccl backends) and drive ShardedGM end to end:
the rank-0 ncclUniqueId broadcast, the library's own RCCL communicator
(transport="rccl") or the torch.distributed all-reduce callback
(transport="torch"), row-major and panel inputs, gm2 and Philox gm — against
the unsharded call.  The two-rank run lives in tools/sharded_2rank.py (torchrun,
both ranks on one GPU over gloo; log in profiles/).
"""
import socket

import pytest
import torch
import torch.distributed as dist

from conftest import rel_l2

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(params=["gloo", "nccl"])
def world1(request):
    """An in-process world of size 1 on cuda:0."""
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    kw = {"device_id": dev} if request.param == "nccl" else {}
    # a port found free can be taken by another socket before the store binds it
    # (EADDRINUSE seen once on the box): take a fresh one then
    for attempt in range(5):
        try:
            dist.init_process_group(request.param,
                                    init_method=f"tcp://127.0.0.1:{_free_port()}",
                                    rank=0, world_size=1, **kw)
            break
        except dist.DistNetworkError:
            if attempt == 4:
                raise
    try:
        yield request.param
    finally:
        dist.destroy_process_group()


def _fill(K, d, B, seed=20211):
    import byzantine_aircomp_amd as bz
    ctx = bz.context()
    s = torch.cuda.current_stream().cuda_stream
    X = torch.empty(K, d, device="cuda")
    bz._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, B, 0.0, 0.05,
                                              0.25, 0.5, seed, s), "fill")
    g0 = torch.empty(d, device="cuda")
    bz._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, seed + 1, s),
                  "fill")
    return X, g0


@pytest.mark.parametrize("transport", ["rccl", "torch"])
@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_sharded_gm2_world1(world1, transport, layout):
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.sharded import ShardedGM
    K, d = 1000, 200_000                  # the C3 recipe and tile (K <= 1024), narrower
    X, g0 = _fill(K, d, 200)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": g0}
    want = bz.gm2(X, dict(opts))
    n = bz.aggregators.last_result.iters
    sg = ShardedGM(d, transport=transport)
    try:
        assert (sg.lo, sg.hi) == (0, d) and sg.world == 1
        Xin = bz.ClientPanels.from_rows(X) if layout == "panels" else X
        got = sg.gm2(Xin, dict(opts))
        torch.cuda.synchronize()
        res = sg.last_result
    finally:
        sg.close()
    assert res.algo == "stream" and res.converged
    assert abs(res.iters - n) <= 1
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


@pytest.mark.parametrize("transport", ["rccl", "torch"])
@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_sharded_gram_world1(world1, transport, layout):
    """AUTO at K <= 256 on a d_total >= 2^18 update: the Gram path's two all-reduces
    (G, then the guard's sums) through the process group."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.sharded import ShardedGM
    K, d = 256, 1 << 19
    X, g0 = _fill(K, d, 51)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": g0}
    want = bz.gm2(X, dict(opts, algo="stream"))
    n = bz.aggregators.last_result.iters
    sg = ShardedGM(d, transport=transport)
    try:
        Xin = bz.ClientPanels.from_rows(X) if layout == "panels" else X
        got = sg.gm2(Xin, dict(opts))
        torch.cuda.synchronize()
        res = sg.last_result
    finally:
        sg.close()
    assert res.algo == "gram" and res.guard == "accepted"
    assert abs(res.iters - n) <= 1
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-5


@pytest.mark.parametrize("transport", ["rccl", "torch"])
@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_sharded_gm_philox_world1(world1, transport, layout):
    """AirComp gm with on-device Philox draws: channel per (iteration, client),
    noise per (iteration, GLOBAL column) — the sharded call reproduces the
    unsharded one's draws."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.sharded import ShardedGM
    K, d = 300, 40_000
    X, g0 = _fill(K, d, 60, seed=77)
    opts = {"maxiter": 30, "tol": 1e-5, "guess": g0, "noise_var": 1e-2, "seed": 4242}
    want = bz.gm(X, dict(opts, algo="stream"))
    sg = ShardedGM(d, transport=transport)
    try:
        Xin = bz.ClientPanels.from_rows(X) if layout == "panels" else X
        got = sg.gm(Xin, dict(opts))
        torch.cuda.synchronize()
        res = sg.last_result
    finally:
        sg.close()
    assert res.iters == 30
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


@pytest.mark.parametrize("transport", ["rccl", "torch"])
def test_sharded_gm_rows_staged_world1(world1, transport):
    """Sharded AirComp gm on rows over >= 64 passes on a large shard streams from the
    context's panel copy (api.hip): the same result as the unsharded row-major passes."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.sharded import ShardedGM
    K, d = 300, 65_536
    X, g0 = _fill(K, d, 60, seed=78)
    opts = {"maxiter": 64, "tol": 1e-5, "guess": g0, "noise_var": 1e-2, "seed": 4243}
    want = bz.gm(X, dict(opts, algo="stream"))
    sg = ShardedGM(d, transport=transport)
    try:
        got = sg.gm(X, dict(opts))
        torch.cuda.synchronize()
        res = sg.last_result
    finally:
        sg.close()
    assert (res.iters, res.algo) == (64, "stream")
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


def test_sharded_requires_guess_and_seed(world1):
    from byzantine_aircomp_amd.sharded import ShardedGM
    sg = ShardedGM(1024, transport="torch")
    try:
        X = torch.zeros(8, 1024, device="cuda")
        with pytest.raises(ValueError):
            sg.gm2(X, {"maxiter": 3})
        with pytest.raises(ValueError):
            sg.gm(X, {"maxiter": 3, "guess": torch.ones(1024, device="cuda")})
        with pytest.raises(ValueError):
            sg.gm2(torch.zeros(8, 1000, device="cuda"), {"guess": torch.ones(1000, device="cuda")})
    finally:
        sg.close()


@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_sharded_pre_oma_world1(world1, layout):
    """ShardedGM gm2 with the fused OMA pre-noise == OMA then the unsharded gm2."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.sharded import ShardedGM
    K, d = 1000, 100_000
    X, g0 = _fill(K, d, 200)
    opts = {"maxiter": 1000, "tol": 1e-5, "guess": g0}
    A = X.clone()
    bz.OMA(A, 1e-2, seed=41)
    want = bz.gm2(A, dict(opts))
    sg = ShardedGM(d, transport="torch")
    try:
        B = bz.ClientPanels.from_rows(X) if layout == "panels" else X.clone()
        got = sg.gm2(B, dict(opts, pre_oma_var=1e-2, pre_oma_seed=41))
        torch.cuda.synchronize()
    finally:
        sg.close()
    Bn = B.to_rows() if layout == "panels" else B
    assert torch.equal(Bn, A)
    assert rel_l2(got.cpu().numpy(), want.cpu().numpy()) <= 1e-6


def iteration_cases():
    """The +-1 inputs above (the device fill restated by oracle/philox_fill.c) for
    tests/test_iteration_wellposed.py."""
    from oracle.philox import fill_clients, fill_normal

    def fill(K, d, B, seed=20211):
        return (torch.from_numpy(fill_clients(K, d, B, 0.0, 0.05, 0.25, 0.5, seed)),
                torch.from_numpy(fill_normal(d, 0.0, 0.01, seed + 1)))
    return [("gm2_world1_1000x200k", lambda: [(*fill(1000, 200_000, 200), 1000, 1e-5)]),
            ("gram_world1_256x2^19", lambda: [(*fill(256, 1 << 19, 51), 1000, 1e-5)])]
