"""The caller side of the aggregation boundary, device-resident.

The reference's federated loop, `SGD` (MNIST_Air_weight.py:226-372), simulates
K clients sequentially and hands the aggregator a CPU matrix built every step
from per-client `.cpu()` copies (M:304, M:341) stacked by `flatten_list`
(M:206-209), then copies the aggregate back parameter by parameter
(M:354-358).  This module is the build's own counterpart:

  * `ClientUpdates` (row f2): one preallocated [K, d] fp32 matrix on the
    model's device; client k's parameters are written straight into row k
    (no host round trip), and the aggregate is copied back into the
    parameters through views — the layout is `flatten_list`'s (client-major,
    `model.parameters()` order).
  * `SGD` (row f4): the same signature, schedule, attacks, RNG consumption and
    outputs as the reference loop, calling any aggregator with the reference's
    `aggregate(wList, options)` contract (ours: `gm2`, `gm`, ...).
  * `run` / `modelFactory` / `calculateAccuracy` / `getVarience`: the driver
    pieces needed to produce records with the reference's keys and titles, so
    draw.ipynb-style plots read them unchanged.

Reference behaviours kept on purpose (pinned by tests/golden e2e fixtures):
  * `model.state_dict()` aliases the parameters, so the reference's
    "snapshot / recovery" around each client (M:290, M:343) restores nothing:
    client k starts from client k-1's updated model, and the aggregator's guess
    (M:349) is the model after the last client.
  * classflip relabels y -> (C-1) - y as an integer (torch 1.1 semantics of
    `9.0 - targets`, M:320; EMNIST: 61 - y); dataflip feeds 1 - x (M:326);
    weightflip rewrites the last B rows as -w - 2*sum(honest)/B (M:380-383).
  * OMA pre-noise is applied iff the aggregator is not `gm` and a variance is
    given (M:351-352).
"""
from __future__ import annotations

import os
import pickle
import random
import sys
import time

import numpy as np
import torch
import torch.nn as nn

__all__ = ["ClientUpdates", "SGD", "run", "modelFactory", "MLP", "setup_seed",
           "calculateAccuracy", "getVarience", "classflip", "dataflip", "weightflip"]


# ---- small pieces with the reference's semantics -------------------------------

def setup_seed(seed):
    """M:30-37."""
    torch.manual_seed(seed)
    torch.cuda.manual_seed(seed)
    torch.cuda.manual_seed_all(seed)
    np.random.seed(seed)
    random.seed(seed)
    torch.backends.cudnn.benchmark = False
    torch.backends.cudnn.deterministic = True


class MLP(nn.Module):
    """The reference's linear model (M:53-61): 784 -> 10 (MNIST) or 784 -> 62 (EMNIST)."""

    def __init__(self, input_size=784, output_size=10):
        super().__init__()
        self.linear = nn.Linear(input_size, output_size)

    def forward(self, x):
        return self.linear(x.view(x.size(0), -1))


def _init_weights(m):
    # M:92-95: xavier-normal with the ReLU gain, bias 0.01
    if isinstance(m, (nn.Conv2d, nn.Linear)):
        nn.init.xavier_normal_(m.weight, gain=nn.init.calculate_gain("relu"))
        nn.init.constant_(m.bias, 0.01)


def modelFactory(SEED=None, num_classes=10):  # noqa: N802 - reference name (M:98)
    if SEED is not None:
        setup_seed(SEED)
    model = MLP(28 * 28, num_classes)
    model.apply(_init_weights)
    return model


def calculateAccuracy(model, loss_func, loader, device):  # noqa: N802 - M:106-125
    loss_sum, correct, total = 0.0, 0, 0
    with torch.no_grad():
        for xb, yb in loader:
            xb, yb = xb.to(device), yb.to(device)
            out = model(xb)
            loss_sum += loss_func(out, yb).item() * len(yb)
            correct += (out.argmax(dim=1) == yb).sum().item()
            total += len(yb)
    return loss_sum / total, correct / total


def getVarience(w_local, honestSize):  # noqa: N802 - M:127-129
    """Mean over the honest rows of ||x_k - honest mean||^2.  On the device (a CUDA
    fp32 [K, d] matrix or ClientPanels) it is ONE streaming pass of the HIP kernel
    gm_honest_variance_f32 (fp64 sums); a CPU matrix (the reference loop's own
    tensors) keeps the reference's torch expression."""
    from .panels import ClientPanels
    if isinstance(w_local, ClientPanels) or (w_local.is_cuda and w_local.dtype == torch.float32):
        from .aggregators import honest_variance
        return honest_variance(w_local, honestSize)
    h = w_local[:honestSize]
    return torch.mean(((h - h.mean(dim=0)) ** 2).sum(dim=1))


def classflip(messages, byzantinesize):
    """The flip itself happens on the labels inside the loop (M:317-323)."""


def dataflip(messages, byzantinesize):
    """The flip itself happens on the inputs inside the loop (M:324-330)."""


def weightflip(messages, byzantinesize):
    """M:380-383, on the device matrix: the last B rows become -w - 2 * sum(honest) / B.
    On ClientPanels ([npan][K][W]) the same per-column rewrite, panel by panel: the
    honest sum runs over each panel's first K - B rows (the padding columns >= d hold 0
    in every row, so they stay 0)."""
    from .panels import ClientPanels
    if isinstance(messages, ClientPanels):
        D = messages.data
        honest_sum = D[:, :-byzantinesize, :].sum(dim=1, keepdim=True)
        D[:, -byzantinesize:, :].mul_(-1).add_(honest_sum / byzantinesize, alpha=-2)
        return
    honest_sum = messages[:-byzantinesize].sum(dim=0)
    messages[-byzantinesize:].mul_(-1).add_(honest_sum / byzantinesize, alpha=-2)


def _oma_host(message, noise_var):
    """OMA (M:385-394) on a CPU matrix, with the reference's own torch expression and
    draw order (the device paths are aggregators.OMA / the fused gm2 pre-noise)."""
    K, d = message.shape
    sd = noise_var ** 0.5
    h_re = torch.normal(torch.zeros(K, 1), 2 ** -0.5)
    h_im = torch.normal(torch.zeros(K, 1), 2 ** -0.5)
    n_re = torch.normal(torch.zeros(K, d), sd)
    n_im = torch.normal(torch.zeros(K, d), sd)
    message.add_((h_re * n_re + h_im * n_im) / (h_re ** 2 + h_im ** 2))


# ---- device-resident client packing (row f2) --------------------------------------

class ClientUpdates:
    """K client parameter vectors, resident on the model's device.

    layout="rows": a [K, d] matrix (flatten_list's stack, M:206-209), row k written
    in place.  layout="panels": a ClientPanels — the same values in the panel layout
    the streaming pass reads contiguously (the C3 headline's input), client k
    scattered into it by `store` (one kernel-free strided copy per client); gm / gm2
    and OMA take it directly."""

    def __init__(self, model: nn.Module, K: int, device=None, layout: str = "rows"):
        self.params = list(model.parameters())
        self.d = sum(p.numel() for p in self.params)
        dev = device if device is not None else self.params[0].device
        if layout not in ("rows", "panels"):
            raise ValueError(f"layout must be 'rows' or 'panels' (got {layout!r})")
        self.layout = layout
        if layout == "panels":
            from .panels import ClientPanels
            self.X = ClientPanels(K, self.d, device=dev)
            self._buf = torch.empty(self.d, dtype=torch.float32, device=dev)
        else:
            self.X = torch.empty(K, self.d, dtype=torch.float32, device=dev)

    def flat(self, out=None):
        """The model's parameters as one vector (flatten_list's row layout)."""
        return torch.cat([p.detach().reshape(-1) for p in self.params], out=out)

    def store(self, k: int):
        if self.layout == "panels":
            self.X.store(k, self.flat(out=self._buf))
        else:
            self.flat(out=self.X[k])

    def load(self, vector: torch.Tensor):
        """Copy an aggregate back into the parameters (M:354-358) through views."""
        off = 0
        vector = vector.to(self.params[0].device)
        with torch.no_grad():
            for p in self.params:
                n = p.numel()
                p.copy_(vector[off:off + n].view_as(p))
                off += n


class _ClientChain:
    """The fused client steps (clients.hip, gm_client_chain_f32): the training set on the
    device once, each step's batch indices from the reference's own samplers."""

    ATTACK = {None: 0, "classflip": 1, "dataflip": 2, "weightflip": 0}

    @classmethod
    def make(cls, model, loss_func, train_dataset, cuts, batch, num_classes, device, mode):
        if mode is False or device is None or torch.device(device).type != "cuda":
            if mode is True:
                raise ValueError("client_kernel=True needs a CUDA device")
            return None
        why = cls._unsupported(model, loss_func, train_dataset, batch, num_classes)
        if why:
            if mode is True:
                raise ValueError(f"client_kernel=True: {why}")
            return None
        return cls(model, train_dataset, cuts, batch, num_classes, torch.device(device))

    @staticmethod
    def _linear(model):
        m = model.module if isinstance(model, nn.DataParallel) else model
        return m.linear if isinstance(m, MLP) else None

    @classmethod
    def _unsupported(cls, model, loss_func, ds, batch, num_classes):
        lin = cls._linear(model)
        if lin is None or lin.bias is None:
            return "the model is not the reference's MLP (one nn.Linear with bias)"
        if not (isinstance(loss_func, nn.CrossEntropyLoss) and loss_func.reduction == "mean"
                and loss_func.weight is None and loss_func.label_smoothing == 0.0):
            return "the loss is not CrossEntropyLoss(reduction='mean')"
        if not isinstance(ds, torch.utils.data.TensorDataset) or len(ds.tensors) != 2:
            return "the training set is not a TensorDataset(x, y)"
        F, C = lin.in_features, lin.out_features
        if C != num_classes or not (1 <= F <= 832 and 1 <= C <= 64 and 1 <= batch <= 64):
            return f"unsupported shape (F={F}, C={C}, batch={batch})"
        if lin.weight.dtype != torch.float32:
            return "fp32 parameters only"
        x, y = ds.tensors
        # the kernel reads F features per sample row and trains on labels in [0, C): the
        # torch loop raises on either mismatch, so the kernel path must not run silently
        if x.dim() < 1 or len(x) == 0 or x[0].numel() != F:
            return f"samples of {x[0].numel() if len(x) else 0} features, the model takes {F}"
        if y.dim() != 1 or len(y) != len(x) or y.dtype.is_floating_point \
                or int(y.min()) < 0 or int(y.max()) >= C:
            return f"labels must be integers in [0, {C}), one per sample"
        return None

    def __init__(self, model, ds, cuts, batch, num_classes, device):
        from . import _lib
        from .aggregators import context
        self.lib, self.ctx = _lib.load(), context(device)
        self.lin = self._linear(model)
        x, y = ds.tensors
        self.x = x.reshape(x.shape[0], -1).to(device, torch.float32).contiguous()
        self.y = y.to(device, torch.int64).contiguous()
        self.F, self.C, self.B = self.lin.in_features, self.lin.out_features, batch
        self.cuts = torch.tensor(cuts[:-1], dtype=torch.int32).unsqueeze(1)
        self.device = device

    @staticmethod
    def draw(streams):
        """One step's batch indices: the samplers' index lists, drawn in client order (a
        RandomSampler seeds its generator from the global one at its first draw, M:260-270;
        later draws touch only its own generator)."""
        return torch.tensor([s._next_index() for s in streams], dtype=torch.int32)

    def step(self, local, clients, honest, attack_name, gamma, wd):
        from . import _lib
        from .aggregators import _stream_ptr
        K = local.shape[0] if local.dim() == 2 else -1
        if local.shape != (K, self.B):
            raise RuntimeError("client batches must be full batches of batchSize samples")
        idx = (local + self.cuts).to(self.device, non_blocking=True)
        Wt, bt = self.lin.weight, self.lin.bias
        if not (Wt.is_contiguous() and bt.is_contiguous()):
            raise RuntimeError("the model's weight and bias must be contiguous")
        X = clients.X
        if clients.layout == "panels":
            buf, ldx, lay = X.data, X.panel_stride, _lib.GM_LAYOUT_PANELS
        else:
            buf, ldx, lay = X, X.stride(0), _lib.GM_LAYOUT_ROWS
        with torch.cuda.device(self.device):
            _lib.check(self.lib.gm_client_chain_f32(
                self.ctx.handle, self.x.data_ptr(), self.F, self.y.data_ptr(), self.F, self.C,
                idx.data_ptr(), K, self.B, honest, self.ATTACK.get(attack_name, 0), float(gamma),
                float(wd), Wt.data_ptr(), bt.data_ptr(), buf.data_ptr(), ldx, lay,
                _stream_ptr(self.device)), "gm_client_chain_f32")


# ---- the federated loop (row f4) ---------------------------------------------------

def _log(*k):
    print(time.strftime("[%m-%d %H:%M:%S] ", time.localtime()), *k)
    sys.stdout.flush()


def SGD(model, gamma, aggregate, weight_decay, noise_var=None, honestSize=0,  # noqa: N802
        byzantineSize=0, attack=None, rounds=10, displayInterval=1000, SEED=None,
        fixSeed=False, loss_func=None, train_dataset=None, validate_dataset=None, device=None,
        batchSize=None, num_classes=10, verbose=True, layout="rows", eval_train=True,
        client_kernel="auto", **kw):
    """Federated SGD with K = honest + Byzantine simulated clients (M:226-372).
    layout="panels" keeps the client matrix in the panel layout (every aggregator).
    client_kernel="auto": on a GPU, with the reference's MLP, CrossEntropyLoss and a
    TensorDataset, the K client steps of a federated step run as ONE HIP kernel
    (gm_client_chain_f32) instead of K host-driven forward/backward passes; True
    requires it, False keeps the per-client torch loop.
    EMNIST_Air_weight.py's variant: num_classes=62 (its MLP(784, 62) and 61 - y
    relabel, E:101, E:321) and eval_train=False (train loss / accuracy recorded as
    0, 0, E:273-274, E:364-365)."""
    def train_eval():
        return calculateAccuracy(model, loss_func, train_all, device) if eval_train else (0, 0)
    assert byzantineSize == 0 or attack is not None
    assert honestSize != 0
    if fixSeed:
        setup_seed(SEED)
    K = honestSize + byzantineSize
    device = device or torch.device("cpu")
    DL = torch.utils.data.DataLoader

    # contiguous data shards, one per client (M:238-239, M:253)
    n = len(train_dataset)
    cuts = [(i * n) // K for i in range(K + 1)]
    shards = [torch.utils.data.Subset(train_dataset, range(cuts[i], cuts[i + 1])) for i in range(K)]
    train_all = DL(dataset=train_dataset, batch_size=batchSize, pin_memory=True, shuffle=False)
    val_all = DL(dataset=validate_dataset, batch_size=batchSize, pin_memory=True, shuffle=False)
    draws = rounds * displayInterval * batchSize
    samplers = [torch.utils.data.sampler.RandomSampler(s, num_samples=draws, replacement=True)
                for s in shards]
    streams = [iter(DL(dataset=shards[i], batch_size=batchSize, sampler=samplers[i]))
               for i in range(K)]

    tl, ta = train_eval()
    vl, va = calculateAccuracy(model, loss_func, val_all, device)
    paths = {"train_loss": [tl], "train_acc": [ta], "val_loss": [vl], "val_acc": [va], "var": []}
    if verbose:
        _log(f"[0/{rounds}] train: loss={tl:.4f} acc={ta:.4f} val: loss={vl:.4f} acc={va:.4f}")

    attack_name = attack.__name__ if attack is not None else None
    clients = ClientUpdates(model, K, layout=layout)
    params = clients.params
    chain = _ClientChain.make(model, loss_func, train_dataset, cuts, batchSize, num_classes,
                              device, client_kernel)
    is_gm = aggregate.__name__ == "gm"
    if noise_var is not None and not is_gm:
        from . import aggregators as _agg
        from .aggregators import OMA
        # our gm2 takes the pre-noise inside its first streaming pass (options
        # pre_oma_var: the same draws, seed drawn from torch's generator as OMA's is)
        fuse_oma = aggregate is _agg.gm2 and _agg._noise_source({}) == _agg._lib.GM_NOISE_PHILOX
    steps_left = rounds * displayInterval
    nxt = None
    for r in range(rounds):
        for _ in range(displayInterval):
            if chain is not None:
                # the K clients' steps as one kernel (clients.hip): the same batches (the
                # samplers' index streams, drawn in client order), the same chain.  The
                # next step's indices are drawn while the kernel and the aggregation run:
                # the samplers are seeded by the first step's draws, so a later draw uses
                # only its own generator and drawing it early changes no random stream
                cur = nxt if nxt is not None else chain.draw(streams)
                chain.step(cur, clients, honestSize, attack_name, gamma, weight_decay)
                steps_left -= 1
                nxt = chain.draw(streams) if steps_left > 0 else None
            for node in (range(K) if chain is None else ()):
                xb, yb = next(streams[node])
                xb, yb = xb.to(device), yb.to(device)
                if node >= honestSize and attack_name == "classflip":
                    yb = (num_classes - 1) - yb          # integer relabel (M:320)
                elif node >= honestSize and attack_name == "dataflip":
                    xb = 1.0 - xb                         # M:326
                loss = loss_func(model(xb), yb)
                model.zero_grad()
                loss.backward()
                with torch.no_grad():
                    for p in params:                      # M:302-303 / M:339-340
                        p.add_(p.grad + weight_decay * p, alpha=-gamma)
                clients.store(node)                       # row `node`, on the device
            X = clients.X
            if attack is not None:
                attack(X, byzantineSize)
            options = {"maxiter": 1000, "tol": 1e-5, "eta": 1, "noise_var": noise_var,
                       "guess": clients.flat(), "honestSize": honestSize}     # M:349-350
            if noise_var is not None and not is_gm:
                if X.device.type == "cpu":
                    _oma_host(X, noise_var)               # M:351-352 on a CPU matrix
                elif fuse_oma:
                    options["pre_oma_var"] = noise_var    # M:351-352, fused into gm2
                else:
                    OMA(X, noise_var)                     # M:351-352
            clients.load(aggregate(X, options))           # M:353-358
        paths["var"].append(getVarience(clients.X, honestSize).cpu())
        tl, ta = train_eval()
        vl, va = calculateAccuracy(model, loss_func, val_all, device)
        for key, v in (("train_loss", tl), ("train_acc", ta), ("val_loss", vl), ("val_acc", va)):
            paths[key].append(v)
        if verbose:
            _log(f"[{r + 1}/{rounds}] train: loss={tl:.4f} acc={ta:.4f} "
                 f"val: loss={vl:.4f} acc={va:.4f}")
    return (model, paths["train_loss"], paths["train_acc"], paths["val_loss"], paths["val_acc"],
            paths["var"])


def run(optimizer, aggregate, attack, config, noise_var=None, dataSetConfig=None,  # noqa: N803
        recordInFile=True, markOnTitle="", device=None, num_classes=10):
    """Driver with the reference's record format and title naming (M:427-492)."""
    cfg = dict(config)
    if attack is None:
        cfg["byzantineSize"] = 0
    elif isinstance(attack, str):
        attack = {"classflip": classflip, "dataflip": dataflip, "weightflip": weightflip}[attack]
    cfg.update(aggregate=aggregate, attack=attack, noise_var=noise_var)
    model = modelFactory(SEED=cfg["SEED"], num_classes=num_classes)
    if device is not None and device != torch.device("cpu"):
        model = nn.DataParallel(model)   # the reference's class name in titles (NB:25)
    model = model.to(device or torch.device("cpu"))
    attack_name = "baseline" if attack is None else attack.__name__
    title = "{}_{}_{}_{}".format(model.__class__.__name__, optimizer.__name__, attack_name,
                                 aggregate.__name__)
    if noise_var is not None:
        title += "_" + str(noise_var)
    if markOnTitle:
        title += "_" + markOnTitle
    res = optimizer(model, device=device, num_classes=num_classes, **cfg)
    _, tl, ta, vl, va, var = res
    record = dict(dataSetConfig or {})
    for key, val in cfg.items():
        if key in ("train_dataset", "validate_dataset"):
            continue
        record[key] = val.__class__.__name__ if callable(val) else val
    record.update(trainLossPath=tl, trainAccPath=ta, valLossPath=vl, valAccPath=va,
                  variencePath=var)
    if recordInFile:
        os.makedirs(os.path.dirname(cfg["CACHE_DIR"] + title) or ".", exist_ok=True)
        with open(cfg["CACHE_DIR"] + title, "wb") as f:
            pickle.dump(record, f)
    return title, record
