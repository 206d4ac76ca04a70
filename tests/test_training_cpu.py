"""Host logic of the training-loop counterpart (row f4), on CPU.

With the CPU oracle standing in for the aggregator, the build's `SGD`
(byzantine_aircomp_amd/training.py) must reproduce the reference's own loop
bit for bit on the golden end-to-end fixtures: data sharding and sampling, RNG
consumption, the integer classflip, the parameter update, the aliasing
"snapshot", the guess, the OMA gate and the records.  (The GPU variant of this
test, tests/test_gpu_training.py, swaps in the HIP aggregators.)
"""
import numpy as np
import pytest
import torch

from conftest import golden_case
from oracle import aggregators as orc
from test_gpu_training import synthetic_mnist


def _as_aggregator(name):
    fn = {"gm2": lambda w, o={}: orc.gm2(w, o)[0], "gm": lambda w, o={}: orc.gm(w, o)[0]}[name]
    fn.__name__ = name
    return fn


@pytest.mark.parametrize("agg_name", ["gm2", "gm"])
def test_sgd_counterpart_bit_exact_with_reference(agg_name):
    from byzantine_aircomp_amd import training as T
    meta, arr = golden_case(f"e2e_sgd_classflip_{agg_name}")
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_mnist(602, 500))
    model = T.modelFactory(SEED=2021)
    res = T.SGD(model, gamma=1e-2, aggregate=_as_aggregator(agg_name), weight_decay=0.0,
                noise_var=meta["noise_var"], honestSize=45, byzantineSize=5,
                attack=T.classflip, rounds=2, displayInterval=2, SEED=2021, fixSeed=True,
                loss_func=torch.nn.CrossEntropyLoss(), train_dataset=tr, validate_dataset=va,
                device=torch.device("cpu"), batchSize=50, verbose=False)
    m, tl, ta, vl, vacc, var = res
    w = torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
    assert np.array_equal(w, arr["weights"])
    assert tl == meta["trainLossPath"] and vl == meta["valLossPath"]
    assert ta == meta["trainAccPath"] and vacc == meta["valAccPath"]
    assert [float(v) for v in var] == meta["variencePath"]


def synthetic_emnist(seed, n, classes=62):
    # same recipe as tests/golden/make_golden.py (synthetic_emnist)
    proto = np.random.default_rng(700).standard_normal((classes, 1, 28, 28)).astype(np.float32)
    r = np.random.default_rng(seed)
    y = r.integers(0, classes, n).astype(np.int64)
    x = (proto[y] + 2.0 * r.standard_normal((n, 1, 28, 28))).astype(np.float32)
    return torch.from_numpy(x), torch.from_numpy(y)


@pytest.mark.parametrize("agg_name", ["gm2", "gm"])
def test_sgd_counterpart_bit_exact_with_emnist_reference(agg_name):
    """EMNIST_Air_weight.py's loop: 62 classes (d = 48,670), the 61 - y flip
    (E:321) and no train-set evaluation (E:273-274, E:364-365)."""
    from byzantine_aircomp_amd import training as T
    meta, arr = golden_case(f"e2e_emnist_classflip_{agg_name}")
    tr = torch.utils.data.TensorDataset(*synthetic_emnist(701, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_emnist(702, 500))
    model = T.modelFactory(SEED=2021, num_classes=62)
    res = T.SGD(model, gamma=1e-2, aggregate=_as_aggregator(agg_name), weight_decay=0.0,
                noise_var=meta["noise_var"], honestSize=45, byzantineSize=5,
                attack=T.classflip, rounds=2, displayInterval=2, SEED=2021, fixSeed=True,
                loss_func=torch.nn.CrossEntropyLoss(), train_dataset=tr, validate_dataset=va,
                device=torch.device("cpu"), batchSize=50, verbose=False, num_classes=62,
                eval_train=False)
    m, tl, ta, vl, vacc, var = res
    w = torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
    assert w.size == meta["d"] == 48_670
    assert np.array_equal(w, arr["weights"])
    assert tl == meta["trainLossPath"] == [0, 0, 0] and ta == meta["trainAccPath"]
    assert vl == meta["valLossPath"] and vacc == meta["valAccPath"]
    assert [float(v) for v in var] == meta["variencePath"]


def test_weightflip_on_device_matrix_semantics():
    from byzantine_aircomp_amd import training as T
    g = torch.Generator().manual_seed(3)
    X = torch.randn(10, 33, generator=g)
    ref = X.clone()
    s = torch.sum(ref[0:-3], dim=0)                 # M:381-383
    ref[-3:].mul_(-1)
    ref[-3:].add_(s / 3, alpha=-2)
    T.weightflip(X, 3)
    assert torch.equal(X, ref)


def test_run_writes_reference_record(tmp_path):
    import pickle
    from byzantine_aircomp_amd import training as T
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 400))
    va = torch.utils.data.TensorDataset(*synthetic_mnist(602, 100))
    cfg = {"honestSize": 8, "byzantineSize": 2, "rounds": 1, "displayInterval": 1,
           "weight_decay": 0.0, "fixSeed": True, "SEED": 2021, "batchSize": 50, "shuffle": True,
           "gamma": 1e-2, "CACHE_DIR": str(tmp_path) + "/mnist_K10_B2_",
           "train_dataset": tr, "validate_dataset": va,
           "loss_func": torch.nn.CrossEntropyLoss()}
    title, rec = T.run(T.SGD, _as_aggregator("gm2"), "classflip", cfg,
                       dataSetConfig={"name": "mnist", "dataSet": "mnist",
                                      "dataSetSize": 400, "maxFeature": 784},
                       device=torch.device("cpu"))
    assert title == "MLP_SGD_classflip_gm2"              # M:446-451 naming
    with open(cfg["CACHE_DIR"] + title, "rb") as f:
        saved = pickle.load(f)                           # our own file
    for key in ("trainLossPath", "trainAccPath", "valLossPath", "valAccPath", "variencePath",
                "honestSize", "byzantineSize", "aggregate", "attack", "name"):
        assert key in saved
    assert saved["aggregate"] == "function" and len(saved["valLossPath"]) == 2


MORE_E2E = [("weightflip", None, "e2e_sgd_weightflip_gm2"), ("dataflip", None, "e2e_sgd_dataflip_gm2"),
            ("classflip", 1e-2, "e2e_sgd_classflip_gm2_var0.01")]


@pytest.mark.parametrize("attack,var,name", MORE_E2E)
def test_sgd_counterpart_bit_exact_more_attacks(attack, var, name):
    """weightflip (M:380-383), dataflip (M:324-330) and `--agg gm2 --var 1e-2` (the OMA
    pre-noise before a non-gm aggregator, M:351-352) through the build's loop with the
    oracle aggregator: bit for bit with the reference's own loop."""
    from byzantine_aircomp_amd import training as T
    meta, arr = golden_case(name)
    assert meta["noise_var"] == var
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 2000))
    va = torch.utils.data.TensorDataset(*synthetic_mnist(602, 500))
    model = T.modelFactory(SEED=2021)
    res = T.SGD(model, gamma=1e-2, aggregate=_as_aggregator("gm2"), weight_decay=0.0,
                noise_var=var, honestSize=45, byzantineSize=5, attack=getattr(T, attack),
                rounds=2, displayInterval=2, SEED=2021, fixSeed=True,
                loss_func=torch.nn.CrossEntropyLoss(), train_dataset=tr, validate_dataset=va,
                device=torch.device("cpu"), batchSize=50, verbose=False)
    m, tl, ta, vl, vacc, vv = res
    w = torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
    assert np.array_equal(w, arr["weights"])
    assert tl == meta["trainLossPath"] and vl == meta["valLossPath"]
    assert ta == meta["trainAccPath"] and vacc == meta["valAccPath"]
    assert [float(v) for v in vv] == meta["variencePath"]


def test_client_kernel_rejects_mismatched_dataset():
    """The fused client kernel (clients.hip) reads F features per sample and trains on
    labels in [0, C): a dataset that the per-client torch loop would reject must not
    reach it — _ClientChain._unsupported names the mismatch."""
    from byzantine_aircomp_amd.training import MLP, _ClientChain
    model = MLP(784, 10)
    loss = torch.nn.CrossEntropyLoss()
    ok = torch.utils.data.TensorDataset(torch.zeros(8, 28, 28), torch.arange(8) % 10)
    assert _ClientChain._unsupported(model, loss, ok, 4, 10) is None
    wide = torch.utils.data.TensorDataset(torch.zeros(8, 29, 28), torch.arange(8) % 10)
    assert "features" in _ClientChain._unsupported(model, loss, wide, 4, 10)
    for y in (torch.arange(8) + 5, torch.arange(8) - 1, torch.zeros(8)):
        bad = torch.utils.data.TensorDataset(torch.zeros(8, 28, 28), y)
        assert "labels" in _ClientChain._unsupported(model, loss, bad, 4, 10)


def test_client_kernel_predrawn_batches_keep_every_random_stream():
    """training.SGD (client kernel) draws step t+1's batch indices while step t's kernel and
    aggregation run.  Only the samplers' first draw touches the global generator (M:260-270:
    RandomSampler seeds its own generator then), so drawing early must leave both the index
    streams and the global stream (OMA seeds, evaluation iterators) exactly as in order."""
    from byzantine_aircomp_amd import training as T
    tr = torch.utils.data.TensorDataset(*synthetic_mnist(601, 400))
    K, B, steps = 5, 10, 6

    def streams():
        n = len(tr)
        cuts = [(i * n) // K for i in range(K + 1)]
        sh = [torch.utils.data.Subset(tr, range(cuts[i], cuts[i + 1])) for i in range(K)]
        return [iter(torch.utils.data.DataLoader(
            sh[i], batch_size=B, sampler=torch.utils.data.RandomSampler(
                sh[i], num_samples=steps * B, replacement=True))) for i in range(K)]

    torch.manual_seed(7)
    st = streams()
    ref, g_ref = [], []
    for _ in range(steps):
        ref.append(T._ClientChain.draw(st))
        g_ref.append(torch.randn(3))                 # a global-generator consumer per step
    torch.manual_seed(7)
    st = streams()
    got, g_got, nxt = [], [], None
    for t in range(steps):
        cur = nxt if nxt is not None else T._ClientChain.draw(st)
        nxt = T._ClientChain.draw(st) if t + 1 < steps else None
        got.append(cur)
        g_got.append(torch.randn(3))
    for a, b in zip(ref, got):
        assert torch.equal(a, b)
    for a, b in zip(g_ref, g_got):
        assert torch.equal(a, b)
