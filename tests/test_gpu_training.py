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
