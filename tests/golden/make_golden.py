"""Generate the golden vectors for the aggregation hot path.

Runs ONLY in the build container, where the reference is mounted read-only at
/root/reference.  It imports the reference's own functions (``gm2``, ``gm``,
``OMA``, ``OMA2``, ``SGD`` from MNIST_Air_weight.py), runs them on seeded
inputs and stores inputs + outputs + the iteration count and last movement as
small fixtures under tests/golden/.  Nothing from the reference is copied: the
fixtures are data, this script is the recipe.

The reference imports torchvision at module level (M:12, M:14), which is not
installed here; empty stand-in modules are placed in ``sys.modules`` before the
import (the script never touches a torchvision symbol: MNIST is not loaded).
Iteration counts are not returned by the reference, so they are captured with
``sys.settrace`` on the first line of the Weiszfeld loop body (M:146 for gm,
M:174 for gm2) and the last ``guess_movement`` on the tol test (M:158, M:182).

Each fixture is also checked against the build's own CPU restatement
(``oracle/aggregators.py``), bit for bit; the script fails if they differ.

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import importlib.util
import json
import math
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/MNIST_Air_weight.py"
REF_EMNIST = "/root/reference/EMNIST_Air_weight.py"
sys.path.insert(0, ROOT)

from oracle import aggregators as orc  # noqa: E402


def load_reference(path=REF, name="byz_reference"):
    sys.dont_write_bytecode = True      # the reference tree is read-only
    for mod_name in ("torchvision", "torchvision.transforms"):
        sys.modules.setdefault(mod_name, types.ModuleType(mod_name))
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class LoopProbe:
    """Counts executions of a loop-body line and records a local at another line."""

    def __init__(self, func_name, body_line, test_line, local="guess_movement"):
        self.func, self.body, self.test, self.local = func_name, body_line, test_line, local
        self.iters, self.moves = 0, []

    def _trace(self, frame, event, arg):
        if frame.f_code.co_name != self.func:
            return None
        if event == "line":
            if frame.f_lineno == self.body:
                self.iters += 1
            elif frame.f_lineno == self.test:
                self.moves.append(float(frame.f_locals[self.local]))
        return self._trace

    def __enter__(self):
        sys.settrace(self._trace)
        return self

    def __exit__(self, *exc):
        sys.settrace(None)


def rng_inputs(seed, K, d, kind, B=0):
    """Seeded client matrices, from numpy's PCG64 (stable across versions)."""
    r = np.random.default_rng(seed)
    if kind == "random":
        X = r.standard_normal((K, d), dtype=np.float32)
        g = (0.1 * r.standard_normal(d)).astype(np.float32)
    elif kind == "sgd":
        # model-scale: x_k = p + 5e-4 z_k for honest rows, Byzantine rows (last
        # B) spread x10 and shifted, guess = p (the current global model, M:349)
        p = (0.07 * r.standard_normal(d)).astype(np.float32)
        Z = r.standard_normal((K, d), dtype=np.float32)
        X = p + 5e-4 * Z
        if B:
            X[K - B:] = p + 5e-3 * Z[K - B:] + 2e-3
        g = p.copy()
    else:
        raise ValueError(kind)
    return X.astype(np.float32), g.astype(np.float32)


def rel_l2(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    ref = load_reference()
    torch.set_num_threads(8)
    manifest = {"reference": "goldenBill/Byzantine_AirComp MNIST_Air_weight.py",
                "torch": torch.__version__, "cases": []}

    def save(name, meta, **arrays):
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)
        meta = dict(meta, name=name, file=name + ".npz")
        manifest["cases"].append(meta)
        print(f"{name:32s} " + ", ".join(f"{k}={v}" for k, v in meta.items()
                                           if k in ("iters", "iters_f64", "last_movement")))

    # ---- gm2 cases (§4.3 a-e) -------------------------------------------------
    gm2_cases = [
        # name, seed, K, d, kind, B, options (without guess), use_guess
        ("gm2_random_K8_d1000", 101, 8, 1000, "random", 0, {"maxiter": 1000, "tol": 1e-5}, True),
        ("gm2_sgd_K50_B5", 102, 50, 7850, "sgd", 5, {"maxiter": 1000, "tol": 1e-5}, True),
        ("gm2_sgd_K50_B10", 103, 50, 7850, "sgd", 10, {"maxiter": 1000, "tol": 1e-5}, True),
        ("gm2_maxiter7_tolneg", 104, 20, 3000, "sgd", 4, {"maxiter": 7, "tol": -1.0}, True),
        ("gm2_defaults", 105, 30, 2000, "sgd", 3, {}, False),
        ("gm2_maxiter0", 106, 5, 64, "random", 0, {"maxiter": 0}, True),
        ("gm2_ragged_K7_d777", 107, 7, 777, "random", 0, {"maxiter": 1000, "tol": 1e-6}, True),
        ("gm2_K1_d513", 108, 1, 513, "random", 0, {"maxiter": 50, "tol": 1e-5}, True),
    ]
    for name, seed, K, d, kind, B, opts, use_guess in gm2_cases:
        X, g = rng_inputs(seed, K, d, kind, B)
        Xt, gt = torch.from_numpy(X.copy()), torch.from_numpy(g.copy())
        o = dict(opts)
        if use_guess:
            o["guess"] = gt
        with LoopProbe("gm2", 174, 182) as pr:
            out = ref.gm2(Xt, o)
        mine, tr = orc.gm2(torch.from_numpy(X.copy()), dict(o))
        assert torch.equal(out, mine), name
        assert tr.iters == pr.iters, (name, tr.iters, pr.iters)
        _, tr64 = orc.gm2_f64(Xt, gt if use_guess else Xt.mean(0),
                              o.get("maxiter", 200), o.get("tol", 1e-5))
        save(name, {"func": "gm2", "K": K, "d": d, "B": B, "options": opts,
                    "guess_supplied": use_guess, "iters": pr.iters,
                    "last_movement": pr.moves[-1] if pr.moves else None,
                    "iters_f64": tr64.iters},
             X=X, guess=g, out=out.numpy())

    # ---- gm2 clamp exercise (§4.3 c): guess equal to a client row + duplicates
    r = np.random.default_rng(109)
    X = r.standard_normal((12, 500), dtype=np.float32) * 0.05
    X[3] = X[7]                         # duplicate rows
    X[4] = X[7]
    g = X[7].copy()                     # guess sits on (three) clients: dist 0 -> 1e-4
    with LoopProbe("gm2", 174, 182) as pr:
        out = ref.gm2(torch.from_numpy(X.copy()), {"maxiter": 1000, "tol": 1e-5,
                                                   "guess": torch.from_numpy(g.copy())})
    mine, tr = orc.gm2(torch.from_numpy(X.copy()), {"maxiter": 1000, "tol": 1e-5,
                                                    "guess": torch.from_numpy(g.copy())})
    assert torch.equal(out, mine) and tr.iters == pr.iters
    save("gm2_clamp_duplicates", {"func": "gm2", "K": 12, "d": 500, "B": 0,
                                  "options": {"maxiter": 1000, "tol": 1e-5},
                                  "guess_supplied": True, "iters": pr.iters,
                                  "last_movement": pr.moves[-1]},
         X=X, guess=g, out=out.numpy())

    # ---- gm (AirComp) cases (§4.3 f): draws replayed from torch.manual_seed --
    gm_cases = [
        ("gm_var1e-2_it1", 201, 50, 7850, 10, 1e-2, 1),
        ("gm_var1e-2_it5", 202, 50, 7850, 10, 1e-2, 5),
        ("gm_var1e-2_it1000", 203, 50, 7850, 10, 1e-2, 1000),
        ("gm_varNone_it5", 204, 50, 7850, 10, None, 5),
        ("gm_varNone_it1000", 205, 50, 7850, 5, None, 1000),
        ("gm_var1e-1_K16_d999", 206, 16, 999, 3, 1e-1, 200),
    ]
    for name, seed, K, d, B, var, maxiter in gm_cases:
        X, g = rng_inputs(seed, K, d, "sgd", B)
        opts = {"maxiter": maxiter, "tol": 1e-5, "noise_var": var}
        torch.manual_seed(seed)
        with LoopProbe("gm", 146, 158) as pr:
            out = ref.gm(torch.from_numpy(X.copy()), dict(opts, guess=torch.from_numpy(g.copy())))
        torch.manual_seed(seed)
        mine, tr = orc.gm(torch.from_numpy(X.copy()), dict(opts, guess=torch.from_numpy(g.copy())))
        assert torch.equal(out, mine), (name, rel_l2(mine, out))
        assert tr.iters == pr.iters
        save(name, {"func": "gm", "K": K, "d": d, "B": B, "options": opts,
                    "guess_supplied": True, "rng_seed": seed, "iters": pr.iters,
                    "last_movement": pr.moves[-1]},
             X=X, guess=g, out=out.numpy())

    # ---- OMA2 standalone ------------------------------------------------------
    r = np.random.default_rng(301)
    M = (r.standard_normal((20, 301)) * 0.3).astype(np.float32)
    for var in (1e-2, None):
        torch.manual_seed(301)
        out = ref.OMA2(torch.from_numpy(M.copy()), P_max=1, noise_var=var, threshold=torch.tensor(0.02))
        torch.manual_seed(301)
        mine = orc.oma2(torch.from_numpy(M.copy()), P_max=1, noise_var=var, threshold=torch.tensor(0.02))
        assert torch.equal(out, mine)
        save(f"oma2_var{var}", {"func": "OMA2", "K": 20, "d": 300, "noise_var": var, "P_max": 1,
                                "threshold": 0.02, "rng_seed": 301},
             message=M, out=out.numpy())

    # ---- OMA (§4.3 g) ---------------------------------------------------------
    for name, seed, K, d, var in (("oma_K50_d1000", 401, 50, 1000, 1e-2),
                                  ("oma_K7_d333_var1e-1", 402, 7, 333, 1e-1)):
        X, _ = rng_inputs(seed, K, d, "sgd", 0)
        A = torch.from_numpy(X.copy())
        torch.manual_seed(seed)
        ref.OMA(A, var)
        B_ = torch.from_numpy(X.copy())
        torch.manual_seed(seed)
        orc.oma_(B_, var)
        assert torch.equal(A, B_)
        save(name, {"func": "OMA", "K": K, "d": d, "noise_var": var, "rng_seed": seed},
             X=X, out=A.numpy())

    # ---- other aggregators (row f3) ----------------------------------------------
    X, _ = rng_inputs(501, 20, 640, "sgd", 4)
    Xt = torch.from_numpy(X)
    outs = {"mean": ref.mean(Xt), "trimmed_mean": ref.trimmed_mean(Xt),
            "median": ref.median(Xt), "Krum": ref.Krum(Xt, {"honestSize": 16}),
            "variance": ref.getVarience(Xt, 16).reshape(1)}
    assert torch.equal(outs["mean"], orc.mean(Xt))
    assert torch.equal(outs["trimmed_mean"], orc.trimmed_mean(Xt))
    assert torch.equal(outs["median"], orc.median(Xt))
    assert torch.equal(outs["Krum"], orc.krum(Xt, {"honestSize": 16}))
    assert torch.equal(outs["variance"], orc.variance(Xt, 16).reshape(1))
    save("other_aggregators_K20_d640", {"func": "other", "K": 20, "d": 640, "honestSize": 16},
         X=X, **{k: v.numpy() for k, v in outs.items()})

    # ---- end-to-end SGD smoke (§4.3 h) ---------------------------------------------
    e2e(ref, manifest, save)

    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote", len(manifest["cases"]), "cases")


def synthetic_mnist(seed, n):
    proto = np.random.default_rng(600).standard_normal((10, 1, 28, 28)).astype(np.float32)
    r = np.random.default_rng(seed)
    y = r.integers(0, 10, n).astype(np.int64)
    x = (proto[y] + 2.0 * r.standard_normal((n, 1, 28, 28))).astype(np.float32)
    return x, y


def e2e(ref, manifest, save):
    """The reference's own SGD loop (M:226-372) on a synthetic MNIST-shaped set.

    classflip's ``9.0 - targets`` (M:320) is a float under torch>=1.2; the pinned
    torch 1.1 cast it back to int64, so the loss is wrapped with ``.long()``.
    """
    ce = torch.nn.CrossEntropyLoss()
    loss = lambda o, t: ce(o, t.long())  # noqa: E731
    xtr, ytr = synthetic_mnist(601, 2000)
    xva, yva = synthetic_mnist(602, 500)
    for agg, var in (("gm2", None), ("gm", 1e-2)):
        tr = torch.utils.data.TensorDataset(torch.from_numpy(xtr), torch.from_numpy(ytr))
        va = torch.utils.data.TensorDataset(torch.from_numpy(xva), torch.from_numpy(yva))
        model = ref.modelFactory(SEED=2021)
        res = ref.SGD(model, gamma=1e-2, aggregate=getattr(ref, agg), weight_decay=0.0,
                      noise_var=var, honestSize=45, byzantineSize=5,
                      attack=ref.classflip, rounds=2, displayInterval=2, SEED=2021,
                      fixSeed=True, loss_func=loss, train_dataset=tr,
                      validate_dataset=va, device=torch.device("cpu"), batchSize=50)
        m, tl, ta, vl, va_, vp = res
        w = torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
        save(f"e2e_sgd_classflip_{agg}", {
            "func": "SGD", "aggregate": agg, "noise_var": var, "K": 50, "B": 5,
            "rounds": 2, "displayInterval": 2, "SEED": 2021, "batchSize": 50,
            "gamma": 1e-2, "data_seeds": [601, 602], "n_train": 2000, "n_val": 500,
            "trainLossPath": tl, "trainAccPath": ta, "valLossPath": vl,
            "valAccPath": va_, "variencePath": [float(v) for v in vp]},
            weights=w)


def synthetic_emnist(seed, n, classes=62):
    proto = np.random.default_rng(700).standard_normal((classes, 1, 28, 28)).astype(np.float32)
    r = np.random.default_rng(seed)
    y = r.integers(0, classes, n).astype(np.int64)
    x = (proto[y] + 2.0 * r.standard_normal((n, 1, 28, 28))).astype(np.float32)
    return x, y


def e2e_emnist():
    """EMNIST_Air_weight.py's SGD (its MLP(784, 62): d = 48,670; the classflip
    relabel 61 - y, E:321; no train-set evaluation, E:273-274 / E:364-365) on a
    synthetic 62-class EMNIST-shaped set; appended to golden.json
    (`python tests/golden/make_golden.py --emnist`)."""
    ref = load_reference(REF_EMNIST, "byz_reference_emnist")
    torch.set_num_threads(8)
    path = os.path.join(HERE, "golden.json")
    manifest = json.load(open(path))
    manifest["cases"] = [c for c in manifest["cases"] if not c["name"].startswith("e2e_emnist")]
    ce = torch.nn.CrossEntropyLoss()
    loss = lambda o, t: ce(o, t.long())  # noqa: E731  (61.0 - targets is a float, E:321)
    xtr, ytr = synthetic_emnist(701, 2000)
    xva, yva = synthetic_emnist(702, 500)
    for agg, var in (("gm2", None), ("gm", 1e-2)):
        tr = torch.utils.data.TensorDataset(torch.from_numpy(xtr), torch.from_numpy(ytr))
        va = torch.utils.data.TensorDataset(torch.from_numpy(xva), torch.from_numpy(yva))
        model = ref.modelFactory(SEED=2021)
        res = ref.SGD(model, gamma=1e-2, aggregate=getattr(ref, agg), weight_decay=0.0,
                      noise_var=var, honestSize=45, byzantineSize=5,
                      attack=ref.classflip, rounds=2, displayInterval=2, SEED=2021,
                      fixSeed=True, loss_func=loss, train_dataset=tr,
                      validate_dataset=va, device=torch.device("cpu"), batchSize=50)
        m, tl, ta, vl, va_, vp = res
        w = torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
        name = f"e2e_emnist_classflip_{agg}"
        np.savez_compressed(os.path.join(HERE, name + ".npz"), weights=w)
        manifest["cases"].append({
            "func": "SGD", "reference": "EMNIST_Air_weight.py", "aggregate": agg,
            "noise_var": var, "K": 50, "B": 5, "num_classes": 62, "d": int(w.size),
            "rounds": 2, "displayInterval": 2, "SEED": 2021, "batchSize": 50,
            "gamma": 1e-2, "data_seeds": [701, 702], "n_train": 2000, "n_val": 500,
            "trainLossPath": tl, "trainAccPath": ta, "valLossPath": vl,
            "valAccPath": va_, "variencePath": [float(v) for v in vp],
            "name": name, "file": name + ".npz"})
    with open(path, "w") as f:
        json.dump(manifest, f, indent=1)
    print("wrote EMNIST e2e cases")


def e2e_more():
    """More of the reference's SGD (M:226-372) for the loop counterpart (row f4), appended
    to golden.json (`python tests/golden/make_golden.py --e2e-more`): the weightflip and
    dataflip attacks (M:380-383, M:324-330) under gm2, and gm2 with --var 1e-2 (the
    reference's OMA pre-noise before a non-gm aggregator, M:351-352)."""
    ref = load_reference()
    torch.set_num_threads(8)
    path = os.path.join(HERE, "golden.json")
    manifest = json.load(open(path))
    ce = torch.nn.CrossEntropyLoss()
    loss = lambda o, t: ce(o, t.long())  # noqa: E731
    xtr, ytr = synthetic_mnist(601, 2000)
    xva, yva = synthetic_mnist(602, 500)
    for attack, agg, var in (("weightflip", "gm2", None), ("dataflip", "gm2", None),
                             ("classflip", "gm2", 1e-2)):
        name = f"e2e_sgd_{attack}_{agg}" + ("" if var is None else f"_var{var:g}")
        manifest["cases"] = [c for c in manifest["cases"] if c["name"] != name]
        tr = torch.utils.data.TensorDataset(torch.from_numpy(xtr), torch.from_numpy(ytr))
        va = torch.utils.data.TensorDataset(torch.from_numpy(xva), torch.from_numpy(yva))
        model = ref.modelFactory(SEED=2021)
        res = ref.SGD(model, gamma=1e-2, aggregate=getattr(ref, agg), weight_decay=0.0,
                      noise_var=var, honestSize=45, byzantineSize=5,
                      attack=getattr(ref, attack), rounds=2, displayInterval=2, SEED=2021,
                      fixSeed=True, loss_func=loss, train_dataset=tr,
                      validate_dataset=va, device=torch.device("cpu"), batchSize=50)
        m, tl, ta, vl, va_, vp = res
        w = torch.cat([p.detach().flatten() for p in m.parameters()]).numpy()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), weights=w)
        manifest["cases"].append({
            "func": "SGD", "attack": attack, "aggregate": agg, "noise_var": var, "K": 50,
            "B": 5, "rounds": 2, "displayInterval": 2, "SEED": 2021, "batchSize": 50,
            "gamma": 1e-2, "data_seeds": [601, 602], "n_train": 2000, "n_val": 500,
            "trainLossPath": tl, "trainAccPath": ta, "valLossPath": vl,
            "valAccPath": va_, "variencePath": [float(v) for v in vp],
            "name": name, "file": name + ".npz"})
        print("wrote", name)
    with open(path, "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    if "--emnist" in sys.argv:
        e2e_emnist()
    elif "--e2e-more" in sys.argv:
        e2e_more()
    else:
        main()
