"""The reference's other aggregators on the GPU (row f3) vs its golden outputs and the oracle."""
import numpy as np
import pytest
import torch

from conftest import golden_case, rel_l2
from oracle import aggregators as orc

pytestmark = pytest.mark.gpu


def test_golden_other_aggregators():
    import byzantine_aircomp_amd as bz
    meta, arr = golden_case("other_aggregators_K20_d640")
    X = torch.from_numpy(arr["X"]).cuda()
    assert np.array_equal(bz.median(X).cpu().numpy(), arr["median"])          # exact element
    assert np.array_equal(bz.Krum(X, {"honestSize": 16}).cpu().numpy(), arr["Krum"])  # a row
    assert rel_l2(bz.mean(X).cpu().numpy(), arr["mean"]) <= 1e-6
    assert rel_l2(bz.trimmed_mean(X).cpu().numpy(), arr["trimmed_mean"]) <= 1e-6


@pytest.mark.parametrize("K,d", [(1, 5), (2, 100), (7, 333), (50, 7850), (64, 1000), (65, 257),
                                 (256, 300)])
def test_coordinate_aggregators_vs_oracle(K, d):
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K + d)
    X = torch.randn(K, d, generator=g)
    X[:, ::7] = torch.round(X[:, ::7])            # ties in some columns
    Xc = X.cuda()
    assert np.array_equal(bz.median(Xc).cpu().numpy(), orc.median(X).numpy())
    assert rel_l2(bz.mean(Xc).cpu().numpy(), orc.mean(X).numpy()) <= 1e-6
    if K >= 3:
        assert rel_l2(bz.trimmed_mean(Xc).cpu().numpy(), orc.trimmed_mean(X).numpy()) <= 1e-6


@pytest.mark.parametrize("K,honest", [(10, 8), (50, 45), (50, 40), (120, 100)])
def test_krum_vs_oracle(K, honest):
    import byzantine_aircomp_amd as bz
    g = torch.Generator().manual_seed(K * 3 + honest)
    X = 0.05 * torch.randn(K, 2000, generator=g)
    X[honest:] += 0.5 * torch.randn(K - honest, 2000, generator=g)
    out = bz.Krum(X.cuda(), {"honestSize": honest})
    want = orc.krum(X, {"honestSize": honest})
    assert torch.equal(out.cpu(), want)
    assert bz.aggregators.Krum.last_index < honest


def test_other_aggregators_cpu_input_roundtrip():
    import byzantine_aircomp_amd as bz
    X = torch.randn(11, 99)
    assert bz.median(X).device.type == "cpu"
    assert torch.equal(bz.median(X), orc.median(X))
