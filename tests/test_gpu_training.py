"""The device-resident training-loop counterpart (rows f2, f4) vs the reference's
own SGD loop, pinned by the golden end-to-end fixtures (tests/golden: the
reference's SGD, M:226-372, run on a synthetic MNIST-shaped set)."""
import numpy as np
import pytest
import torch

from conftest import golden_case, rel_l2

pytestmark = pytest.mark.gpu


def synthetic_mnist(seed, n):
    # same recipe as tests/golden/make_golden.py
    proto = np.random.default_rng(600).standard_normal((10, 1, 28, 28)).astype(np.float32)
    r = np.random.default_rng(seed)
    y = r.integers(0, 10, n).astype(np.int64)
    x = (proto[y] + 2.0 * r.standard_normal((n, 1, 28, 28))).astype(np.float32)
    return torch.from_numpy(x), torch.from_numpy(y)


def _run(agg_name, device, monkeypatch, layout="rows"):
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import training as T
    meta, arr = golden_case(f"e2e_sgd_classflip_{agg_name}")
    if agg_name == "gm":
        monkeypatch.setenv("BYZ_AIRCOMP_NOISE", "host")   # replay the reference's draws
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_mnist(602, 500))
    model = T.modelFactory(SEED=2021).to(device)
    agg = getattr(bz, agg_name)
    res = T.SGD(model, gamma=1e-2, aggregate=agg, weight_decay=0.0, noise_var=meta["noise_var"],
                honestSize=45, byzantineSize=5, attack=T.classflip, rounds=2, displayInterval=2,
                SEED=2021, fixSeed=True, loss_func=torch.nn.CrossEntropyLoss(),
                train_dataset=tr, validate_dataset=va, device=torch.device(device),
                batchSize=50, verbose=False, layout=layout)
    m, tl, ta, vl, vacc, var = res
    w = torch.cat([p.detach().flatten().cpu() for p in m.parameters()]).numpy()
    return meta, arr, w, tl, ta, vl, vacc, var


@pytest.mark.parametrize("agg_name", ["gm2", "gm"])
def test_loop_with_cpu_model_matches_reference(agg_name, monkeypatch):
    """Model on CPU like the fixture; only the aggregation runs on the GPU."""
    meta, arr, w, tl, ta, vl, vacc, var = _run(agg_name, "cpu", monkeypatch)
    assert rel_l2(w, arr["weights"]) <= 1e-5
    np.testing.assert_allclose(tl, meta["trainLossPath"], rtol=1e-5)
    np.testing.assert_allclose(vl, meta["valLossPath"], rtol=1e-5)
    assert ta == meta["trainAccPath"] and vacc == meta["valAccPath"]
    np.testing.assert_allclose([float(v) for v in var], meta["variencePath"], rtol=1e-4)


@pytest.mark.parametrize("agg_name", ["gm2", "gm"])
def test_loop_device_resident_matches_reference(agg_name, monkeypatch):
    """Model, client matrix and aggregation all on the GPU (no host round trip)."""
    meta, arr, w, tl, ta, vl, vacc, var = _run(agg_name, "cuda", monkeypatch)
    assert rel_l2(w, arr["weights"]) <= 1e-4
    np.testing.assert_allclose(tl, meta["trainLossPath"], rtol=1e-4)
    np.testing.assert_allclose(vl, meta["valLossPath"], rtol=1e-4)


@pytest.mark.parametrize("agg_name", ["gm2", "gm"])
def test_loop_device_resident_panels_matches_reference(agg_name, monkeypatch):
    """The same loop with the client matrix kept in the panel layout (the layout the
    C3 headline streams): stores scatter into panels, OMA / gm / gm2 / getVarience
    read them directly."""
    meta, arr, w, tl, ta, vl, vacc, var = _run(agg_name, "cuda", monkeypatch, layout="panels")
    assert rel_l2(w, arr["weights"]) <= 1e-4
    np.testing.assert_allclose(tl, meta["trainLossPath"], rtol=1e-4)
    np.testing.assert_allclose(vl, meta["valLossPath"], rtol=1e-4)
    np.testing.assert_allclose([float(v) for v in var], meta["variencePath"], rtol=1e-4)


def test_client_updates_panels_equal_rows():
    from byzantine_aircomp_amd import training as T
    m = T.MLP(784, 10).cuda()
    rows, pan = T.ClientUpdates(m, 5), T.ClientUpdates(m, 5, layout="panels")
    for k in range(5):
        with torch.no_grad():
            for p in m.parameters():
                p.add_(0.5 * k)
        rows.store(k)
        pan.store(k)
    assert torch.equal(pan.X.to_rows(), rows.X)


def test_client_updates_layout_is_flatten_list():
    from byzantine_aircomp_amd import training as T
    m = T.MLP(784, 10).cuda()
    cu = T.ClientUpdates(m, 3)
    for k in range(3):
        with torch.no_grad():
            for p in m.parameters():
                p.add_(1.0)
        cu.store(k)
    want = torch.cat([p.detach().flatten() for p in m.parameters()])
    assert torch.equal(cu.X[2], want)
    assert cu.X.shape == (3, 7850) and cu.X.device.type == "cuda"
    cu.load(torch.zeros(7850, device="cuda"))
    assert all(float(p.abs().sum()) == 0 for p in m.parameters())


@pytest.mark.parametrize("agg_name", ["gm2", "gm"])
@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_emnist_loop_device_resident_matches_reference(agg_name, layout, monkeypatch):
    """EMNIST_Air_weight.py's loop (62 classes, d = 48,670, 61 - y, no train-set
    evaluation) with model, client matrix and aggregation on the GPU."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import training as T
    from test_training_cpu import synthetic_emnist
    meta, arr = golden_case(f"e2e_emnist_classflip_{agg_name}")
    if agg_name == "gm":
        monkeypatch.setenv("BYZ_AIRCOMP_NOISE", "host")   # replay the reference's draws
    tr = torch.utils.data.TensorDataset(*synthetic_emnist(701, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_emnist(702, 500))
    model = T.modelFactory(SEED=2021, num_classes=62).cuda()
    res = T.SGD(model, gamma=1e-2, aggregate=getattr(bz, agg_name), weight_decay=0.0,
                noise_var=meta["noise_var"], honestSize=45, byzantineSize=5, attack=T.classflip,
                rounds=2, displayInterval=2, SEED=2021, fixSeed=True,
                loss_func=torch.nn.CrossEntropyLoss(), train_dataset=tr, validate_dataset=va,
                device=torch.device("cuda"), batchSize=50, verbose=False, num_classes=62,
                eval_train=False, layout=layout)
    m, tl, ta, vl, vacc, var = res
    w = torch.cat([p.detach().flatten() for p in m.parameters()]).cpu().numpy()
    assert rel_l2(w, arr["weights"]) <= 1e-4
    np.testing.assert_allclose(vl, meta["valLossPath"], rtol=1e-4)
    np.testing.assert_allclose([float(v) for v in var], meta["variencePath"], rtol=1e-4)


@pytest.mark.parametrize("layout", ["rows", "panels"])
@pytest.mark.parametrize("attack,var,name", [
    ("weightflip", None, "e2e_sgd_weightflip_gm2"), ("dataflip", None, "e2e_sgd_dataflip_gm2"),
    ("classflip", 1e-2, "e2e_sgd_classflip_gm2_var0.01")])
def test_loop_more_attacks_device_resident(attack, var, name, layout, monkeypatch):
    """weightflip (M:380-383: on panels a per-panel rewrite of the last B rows), dataflip
    and `--agg gm2 --var 1e-2` (OMA pre-noise with the reference's replayed draws) with
    model, client matrix and aggregation on the GPU, rows and panels."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import training as T
    meta, arr = golden_case(name)
    if var is not None:
        monkeypatch.setenv("BYZ_AIRCOMP_NOISE", "host")   # the reference's OMA draws
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_mnist(602, 500))
    model = T.modelFactory(SEED=2021).cuda()
    res = T.SGD(model, gamma=1e-2, aggregate=bz.gm2, weight_decay=0.0, noise_var=var,
                honestSize=45, byzantineSize=5, attack=getattr(T, attack), rounds=2,
                displayInterval=2, SEED=2021, fixSeed=True, loss_func=torch.nn.CrossEntropyLoss(),
                train_dataset=tr, validate_dataset=va, device=torch.device("cuda"), batchSize=50,
                verbose=False, layout=layout)
    m, tl, ta, vl, vacc, vv = res
    w = torch.cat([p.detach().flatten() for p in m.parameters()]).cpu().numpy()
    assert rel_l2(w, arr["weights"]) <= 1e-4
    np.testing.assert_allclose(tl, meta["trainLossPath"], rtol=1e-4)
    np.testing.assert_allclose(vl, meta["valLossPath"], rtol=1e-4)
    np.testing.assert_allclose([float(v) for v in vv], meta["variencePath"], rtol=1e-4)


def _chain_reference(x, y, idx, W, b, honest, attack, gamma, wd, C):
    """The reference's client loop body (M:291-343) in float64 torch with autograd:
    client k starts from client k-1's parameters (the aliasing snapshot, M:290/343)."""
    W, b = W.double().clone(), b.double().clone()
    rows = []
    for k in range(idx.shape[0]):
        xb, yb = x[idx[k].long()].double(), y[idx[k].long()].clone()
        if k >= honest and attack == 1:
            yb = (C - 1) - yb
        if k >= honest and attack == 2:
            xb = 1.0 - xb
        Wv, bv = W.clone().requires_grad_(), b.clone().requires_grad_()
        loss = torch.nn.functional.cross_entropy(xb @ Wv.T + bv, yb)
        loss.backward()
        with torch.no_grad():
            W = W - gamma * (Wv.grad + wd * W)
            b = b - gamma * (bv.grad + wd * b)
        rows.append(torch.cat([W.flatten(), b]))
    return torch.stack(rows), W, b


@pytest.mark.parametrize("C", [10, 62])
@pytest.mark.parametrize("attack", [0, 1, 2])
@pytest.mark.parametrize("layout", ["rows", "panels"])
@pytest.mark.parametrize("F", [784, 783])
def test_client_chain_kernel_vs_fp64(C, attack, layout, F):
    """gm_client_chain_f32 (clients.hip) against the loop body in float64: every client's
    row of the client matrix and the final W / b (the last client's, M:349).  F = 784 takes
    the float2 phase-A kernel, odd F the scalar one."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.panels import ClientPanels
    g = torch.Generator().manual_seed(C * 10 + attack)
    n, K, B, honest = 3000, 12, 50, 9
    x = (0.3 * torch.randn(n, F, generator=g)).cuda()
    y = torch.randint(0, C, (n,), generator=g).cuda()
    idx = torch.randint(0, n, (K, B), generator=g, dtype=torch.int32).cuda()
    W0 = (0.05 * torch.randn(C, F, generator=g)).cuda()
    b0 = torch.full((C,), 0.01).cuda()
    d = C * F + C
    want, Ww, bw = _chain_reference(x.cpu(), y.cpu(), idx.cpu(), W0.cpu(), b0.cpu(), honest,
                                    attack, 1e-2, 1e-3, C)
    W, b = W0.clone(), b0.clone()
    if layout == "panels":
        Xp = ClientPanels(K, d)
        buf, ldx, lay = Xp.data, Xp.panel_stride, _lib.GM_LAYOUT_PANELS
    else:
        Xr = torch.full((K, d + 3), float("nan"), device="cuda")
        buf, ldx, lay = Xr, d + 3, _lib.GM_LAYOUT_ROWS
    ctx = bz.context()
    _lib.check(ctx.lib.gm_client_chain_f32(ctx.handle, x.data_ptr(), F, y.data_ptr(), F, C,
                                           idx.data_ptr(), K, B, honest, attack, 1e-2, 1e-3,
                                           W.data_ptr(), b.data_ptr(), buf.data_ptr(), ldx, lay,
                                           torch.cuda.current_stream().cuda_stream), "chain")
    torch.cuda.synchronize()
    got = Xp.to_rows() if layout == "panels" else Xr[:, :d]
    assert rel_l2(got.cpu().numpy(), want.numpy()) <= 1e-6
    for k in range(K):
        assert rel_l2(got[k].cpu().numpy(), want[k].numpy()) <= 1e-6, k
    assert rel_l2(W.cpu().numpy(), Ww.numpy()) <= 1e-6
    assert rel_l2(b.cpu().numpy(), bw.numpy()) <= 1e-6


@pytest.mark.parametrize("layout", ["rows", "panels"])
def test_loop_client_kernel_equals_torch_loop(layout):
    """SGD with the fused client steps vs the per-client torch loop on the GPU: the
    same batches (sampler draws in the reference's order) and records to fp32 rounding."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import training as T
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_mnist(602, 500))
    out = []
    for ck in (True, False):
        model = T.modelFactory(SEED=2021).cuda()
        res = T.SGD(model, gamma=1e-2, aggregate=bz.gm2, weight_decay=0.0, honestSize=45,
                    byzantineSize=5, attack=T.classflip, rounds=2, displayInterval=3, SEED=2021,
                    fixSeed=True, loss_func=torch.nn.CrossEntropyLoss(), train_dataset=tr,
                    validate_dataset=va, device=torch.device("cuda"), batchSize=50,
                    verbose=False, layout=layout, client_kernel=ck)
        out.append(res)
    (m1, tl1, _, vl1, _, v1), (m2, tl2, _, vl2, _, v2) = out
    w1 = torch.cat([p.detach().flatten() for p in m1.parameters()]).cpu().numpy()
    w2 = torch.cat([p.detach().flatten() for p in m2.parameters()]).cpu().numpy()
    assert rel_l2(w1, w2) <= 1e-5
    np.testing.assert_allclose(tl1, tl2, rtol=1e-5)
    np.testing.assert_allclose(vl1, vl2, rtol=1e-5)
    np.testing.assert_allclose([float(v) for v in v1], [float(v) for v in v2], rtol=1e-4)
