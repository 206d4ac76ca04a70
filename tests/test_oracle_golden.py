"""Pin the CPU oracle (oracle/aggregators.py) to the reference's golden vectors.

The fixtures were produced by importing the reference itself
(tests/golden/make_golden.py); the oracle must reproduce every one of them bit
for bit, iteration counts included.  CPU only.
"""
import numpy as np
import pytest
import torch

from conftest import golden_case, golden_names
from oracle import aggregators as orc


def _opts(meta, arr):
    o = dict(meta["options"])
    if meta.get("guess_supplied"):
        o["guess"] = torch.from_numpy(arr["guess"].copy())
    return o


@pytest.mark.parametrize("name", golden_names("gm2"))
def test_gm2_bit_exact(name):
    meta, arr = golden_case(name)
    out, tr = orc.gm2(torch.from_numpy(arr["X"].copy()), _opts(meta, arr))
    assert np.array_equal(out.numpy(), arr["out"])
    assert tr.iters == meta["iters"]
    if meta["last_movement"] is not None:
        assert tr.last_movement == pytest.approx(meta["last_movement"], rel=0, abs=0)


@pytest.mark.parametrize("name", golden_names("gm"))
def test_gm_bit_exact(name):
    meta, arr = golden_case(name)
    torch.manual_seed(meta["rng_seed"])
    out, tr = orc.gm(torch.from_numpy(arr["X"].copy()), _opts(meta, arr))
    assert np.array_equal(out.numpy(), arr["out"])
    assert tr.iters == meta["iters"]


@pytest.mark.parametrize("name", golden_names("OMA"))
def test_oma_bit_exact(name):
    meta, arr = golden_case(name)
    X = torch.from_numpy(arr["X"].copy())
    torch.manual_seed(meta["rng_seed"])
    orc.oma_(X, meta["noise_var"])
    assert np.array_equal(X.numpy(), arr["out"])


@pytest.mark.parametrize("name", golden_names("OMA2"))
def test_oma2_bit_exact(name):
    meta, arr = golden_case(name)
    torch.manual_seed(meta["rng_seed"])
    out = orc.oma2(torch.from_numpy(arr["message"].copy()), P_max=meta["P_max"],
                   noise_var=meta["noise_var"], threshold=torch.tensor(meta["threshold"]))
    assert np.array_equal(out.numpy(), arr["out"])


def test_other_aggregators():
    meta, arr = golden_case("other_aggregators_K20_d640")
    X = torch.from_numpy(arr["X"])
    assert np.array_equal(orc.mean(X).numpy(), arr["mean"])
    assert np.array_equal(orc.trimmed_mean(X).numpy(), arr["trimmed_mean"])
    assert np.array_equal(orc.median(X).numpy(), arr["median"])
    assert np.array_equal(orc.krum(X, {"honestSize": 16}).numpy(), arr["Krum"])
    assert np.array_equal(orc.variance(X, 16).reshape(1).numpy(), arr["variance"])


def test_f64_agrees_with_fp32_on_sgd_inputs():
    meta, arr = golden_case("gm2_sgd_K50_B5")
    g64, tr = orc.gm2_f64(torch.from_numpy(arr["X"]), torch.from_numpy(arr["guess"]),
                          meta["options"]["maxiter"], meta["options"]["tol"])
    rel = float((g64 - torch.from_numpy(arr["out"]).double()).norm() / g64.norm())
    assert rel < 1e-6
    assert abs(tr.iters - meta["iters"]) <= 1
