"""Drop-in aggregators backed by libgmagg.so (HIP kernels for gfx950).

The reference resolves its aggregator with ``eval(args.agg)``
(MNIST_Air_weight.py:580) and calls it once per step as
``weight_vector = aggregate(weight_f, options)`` (M:353).  This module provides
functions with the same names, signatures, option keys, defaults and return
semantics, so the reference's training loop can import them in place of its
own:

  ``gm2(wList, options)``  ideal Weiszfeld geometric median      (M:162-184)
  ``gm(wList, options)``   AirComp Weiszfeld, OMA2 every step    (M:131-160, M:396-414)
  ``OMA(message, noise_var)``  in-place per-client pre-noise     (M:385-394)

Semantics kept from the reference:
  * option keys ``maxiter`` (default 200), ``tol`` (1e-5), ``guess`` (default
    the row mean), plus ``noise_var`` (None) and ``P_max`` (1) for ``gm``;
    ``eta`` / ``honestSize`` are ignored, as in the reference;
  * ``maxiter == 0`` returns the ``guess`` object itself;
  * ``wList`` and ``guess`` are not modified (``OMA`` modifies ``message``);
  * the result lives on ``wList.device``: a CPU input is staged to the GPU and
    the aggregate copied back (the reference's hot path runs on CPU tensors);
  * the tol test is on the fp32 movement, returning the NEW iterate.

Extensions (ignored by the reference's loop): options ``noise_source``
(``"device"``: on-device Philox, the default; ``"host"``: the reference's own
``torch.normal`` draws on the CPU generator, in its order, for exact
comparison), ``seed`` (Philox key; drawn from the torch CPU generator when
absent) and ``algo`` (``"auto"``, ``"stream"``, ``"twopass"``, ``"gram"``,
``"gram_f32"``, ``"resident"``).  ``gm2`` / ``gm`` also accept a
``ClientPanels`` (panels.py: the same K x d values in the panel layout the
streaming pass reads as contiguous blocks) in place of the ``[K, d]`` tensor.  The trace of
the last call (iterations, last movement) is in ``last_result``.

There is no CPU path: without a GPU or without libgmagg.so these raise.
"""
from __future__ import annotations

import atexit
import ctypes as C
import math
import os
from dataclasses import dataclass

import torch

from . import _lib
from .panels import ClientPanels

__all__ = ["gm2", "gm", "OMA", "mean", "median", "trimmed_mean", "Krum", "GMResult",
           "last_result", "Context", "context", "honest_variance"]


@dataclass
class GMResult:
    iters: int
    last_movement: float
    converged: bool
    algo: str
    guard: str = "none"      # Gram guard: "none", "accepted", "accepted_floor", "rejected"
    gram_kind: str = ""      # Gram runs: "f16_split", "bf16_split" (f16 range fallback), "f32"
    exchange: str = "none"   # resident runs: "agent" (flat, over XCDs), "xcd_local" (one XCD's
    #                          L2), "xcd_hier" (per-XCD gather, then the 8 XCD sums) or
    #                          "xcd_split" (one hop, own-XCD blocks from L2-kept copies)


last_result: GMResult | None = None
_ALGOS = {"auto": _lib.GM_ALGO_AUTO, "stream": _lib.GM_ALGO_STREAM,
          "twopass": _lib.GM_ALGO_TWOPASS, "gram": _lib.GM_ALGO_GRAM,
          "resident": _lib.GM_ALGO_RESIDENT, "gram_f32": _lib.GM_ALGO_GRAM_F32}
_ALGO_NAMES = {v: k for k, v in _ALGOS.items()}
_GUARD_NAMES = {_lib.GM_GUARD_NONE: "none", _lib.GM_GUARD_ACCEPTED: "accepted",
                _lib.GM_GUARD_REJECTED: "rejected", _lib.GM_GUARD_ACCEPTED_FLOOR: "accepted_floor"}


def _result(res) -> "GMResult":
    return GMResult(res.iters, res.last_movement, bool(res.converged),
                    _ALGO_NAMES.get(res.algo_used, "?"), _GUARD_NAMES.get(res.guard, "?"),
                    {1: "f16_split", 2: "bf16_split", 3: "f32"}.get(res.gram_kind, ""),
                    {1: "agent", 2: "xcd_local", 3: "xcd_hier",
                     4: "xcd_split"}.get(res.exchange, "none"))


class Context:
    """One libgmagg context (device workspace, optional d-shard / RCCL comm)."""

    def __init__(self, device: int):
        self.lib = _lib.load()
        self.device = device
        h = C.c_void_p()
        _lib.check(self.lib.gm_ctx_create(device, C.byref(h)), "gm_ctx_create")
        self.handle = h
        self._keep = []   # ctypes callbacks that must outlive the context

    def set_shard(self, d_total: int, d_offset: int):
        _lib.check(self.lib.gm_ctx_set_shard(self.handle, d_total, d_offset), "gm_ctx_set_shard")

    def set_allreduce(self, fn):
        """fn(dev_ptr:int, count:int, stream:int) -> None; sums doubles in place."""
        def tramp(user, buf, count, stream):
            try:
                fn(buf, count, stream)
                return 0
            except Exception:  # noqa: BLE001 - reported through the status code
                return 1
        cb = _lib.ALLREDUCE_CB(tramp)
        self._keep.append(cb)
        _lib.check(self.lib.gm_ctx_set_allreduce(self.handle, cb, None), "gm_ctx_set_allreduce")

    def init_rccl(self, unique_id: bytes, nranks: int, rank: int):
        buf = C.create_string_buffer(bytes(unique_id), 128)
        _lib.check(self.lib.gm_ctx_init_rccl(self.handle, buf, nranks, rank), "gm_ctx_init_rccl")

    def pass_timing(self, enable: bool):
        """Return (total_ms, launches) of the fused pass since the last call."""
        ms, n = C.c_double(), C.c_int64()
        _lib.check(self.lib.gm_ctx_pass_timing(self.handle, int(enable), C.byref(ms),
                                               C.byref(n)), "gm_ctx_pass_timing")
        return ms.value, n.value

    def close(self):
        """Destroy the context now (workspace, RCCL communicator); idempotent.
        Multi-process callers close before torch.distributed.destroy_process_group()
        rather than leaving the communicator to interpreter teardown."""
        h, self.handle = getattr(self, "handle", None), None
        if h:
            self.lib.gm_ctx_destroy(h)
        for k, v in list(_contexts.items()):
            if v is self:
                del _contexts[k]

    def __del__(self):
        try:
            if getattr(self, "handle", None):
                self.lib.gm_ctx_destroy(self.handle)
        except Exception:  # noqa: BLE001 - interpreter teardown
            pass


_contexts: dict[int, Context] = {}


def close_all():
    """Destroy every per-device context now (workspace, pinned host buffer, events).
    Registered with atexit, so it runs in Py_Finalize — before the C-level exit
    handlers that tear the HIP runtime down — instead of from Context.__del__ during
    interpreter teardown, when the runtime (or a profiler intercepting it) may already
    be finalised."""
    for ctx in list(_contexts.values()):
        ctx.close()


if os.environ.get("GMAGG_ATEXIT_CLOSE", "1") != "0":    # (=0: the round-2 behaviour, A/B)
    atexit.register(close_all)


def context(device: torch.device | int | None = None) -> Context:
    if not torch.cuda.is_available():
        raise RuntimeError("byzantine_aircomp_amd needs a ROCm GPU (torch.cuda.is_available() "
                           "is False); there is no CPU fallback")
    if device is None:
        idx = torch.cuda.current_device()
    elif isinstance(device, int):
        idx = device
    else:
        idx = device.index if device.index is not None else torch.cuda.current_device()
    ctx = _contexts.get(idx)
    if ctx is None:
        ctx = _contexts[idx] = Context(idx)
    return ctx


def _stream_ptr(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


def _stage(t: torch.Tensor) -> torch.Tensor:
    """The GPU tensor the kernels read (a copy if `t` lives on the CPU)."""
    if t.dtype != torch.float32:
        raise TypeError(f"aggregation kernels are fp32 (got {t.dtype})")
    if t.device.type == "cuda":
        return t
    return t.to(torch.device("cuda", torch.cuda.current_device()))


def _rows(X: torch.Tensor):
    """(tensor, ldx) with unit column stride, rows >= d apart."""
    if X.dim() != 2:
        raise ValueError(f"wList must be [K, d] (got {tuple(X.shape)})")
    if X.stride(1) != 1 or X.stride(0) < X.shape[1] or X.shape[0] == 0:
        X = X.contiguous()
    return X, max(X.stride(0), X.shape[1])


def _noise_source(options) -> int:
    src = options.get("noise_source", os.environ.get("BYZ_AIRCOMP_NOISE", "device"))
    if src == "device":
        return _lib.GM_NOISE_PHILOX
    if src == "host":
        return _lib.GM_NOISE_HOST
    raise ValueError(f"noise_source must be 'device' or 'host' (got {src!r})")


def _seed(options) -> int:
    if options.get("seed") is not None:
        return int(options["seed"]) & (2 ** 64 - 1)
    return int(torch.randint(0, 2 ** 62, (1,)).item())


def _host_draws(K: int, d: int, noise_var):
    """The reference's OMA2 draws, in order, on the global CPU generator (M:401-411)."""
    def cb(user, it, hr, hi, n):
        try:
            a = torch.normal(torch.zeros(K), 1 / math.sqrt(2))
            b = torch.normal(torch.zeros(K), 1 / math.sqrt(2))
            C.memmove(hr, a.data_ptr(), 4 * K)
            C.memmove(hi, b.data_ptr(), 4 * K)
            if noise_var is not None:
                z = torch.normal(torch.zeros(d + 1), math.sqrt(noise_var / 2))
                C.memmove(n, z.data_ptr(), 4 * (d + 1))
            return 0
        except Exception:  # noqa: BLE001
            return 1
    return _lib.NOISE_CB(cb)


def _weiszfeld(wList: torch.Tensor, options: dict, aircomp: bool):
    global last_result
    opts = {"maxiter": 200, "tol": 1e-5}
    if aircomp:
        opts.update({"noise_var": None, "P_max": 1})
    opts.update(options or {})
    # pre_oma_var: the reference's OMA(weight_f, var) before a non-gm aggregator
    # (M:351-352), in place on wList, fused into the first streaming pass (pre_oma_seed
    # keys the Philox draws as OMA(..., seed=)).  With the default guess (the column mean
    # of the NOISY rows) it runs as the separate OMA first.
    pre_var = None if aircomp else opts.get("pre_oma_var")
    # (the Philox key is drawn only where Philox draws are made: with host draws OMA
    # replays the reference's torch.normal sequence, which an extra randint would shift)
    pre_seed = opts.get("pre_oma_seed")
    if pre_var is not None and (opts.get("guess") is None or wList.device.type != "cuda"
                                or _noise_source(opts) == _lib.GM_NOISE_HOST):
        # (the reference's own draws are host-side: OMA replays them itself)
        OMA(wList, float(pre_var), noise_source=opts.get("noise_source"), seed=pre_seed)
        pre_var = None
    guess = opts.get("guess")
    if guess is None:
        guess = wList.mean(dim=0)
    maxiter = int(opts["maxiter"])
    if maxiter <= 0:                        # M:145 / M:173 loop body never runs
        if pre_var is not None:
            OMA(wList, float(pre_var), seed=pre_seed)
        last_result = GMResult(0, float("nan"), False, "none")
        return guess
    layout = _lib.GM_LAYOUT_ROWS
    if isinstance(wList, ClientPanels):
        X, ldx, layout = wList.data, wList.panel_stride, _lib.GM_LAYOUT_PANELS
        K, d = wList.shape
    else:
        X = _stage(wList)
        X, ldx = _rows(X)
        K, d = X.shape
    g0 = guess.detach().to(device=X.device, dtype=torch.float32).contiguous()
    if g0.numel() != d:
        raise ValueError(f"guess has {g0.numel()} elements, wList rows have {d}")
    out = torch.empty(d, dtype=torch.float32, device=X.device)
    if d == 0:
        last_result = GMResult(1, 0.0, True, "none")
        return out.to(wList.device)

    o = _lib.GmOpts()
    o.maxiter = maxiter
    o.tol = float(opts["tol"])
    o.eps = 1e-4
    o.mode = _lib.GM_MODE_AIRCOMP if aircomp else _lib.GM_MODE_IDEAL
    o.algo = _ALGOS[opts.get("algo", "auto")]
    o.check_every = int(opts.get("check_every", 0))
    o.layout = layout
    if pre_var is not None:
        o.pre_oma = 1
        o.pre_oma_var = float(pre_var)
        o.pre_oma_seed = _seed({"seed": pre_seed})
    cb = None
    if aircomp:
        var = opts["noise_var"]
        o.has_noise = int(var is not None)
        o.noise_var = float(var) if var is not None else 0.0
        o.P_max = float(opts["P_max"])
        o.noise_source = _noise_source(opts)
        if o.noise_source == _lib.GM_NOISE_HOST:
            cb = _host_draws(K, d, var)
            o.noise_cb = cb
        else:
            o.seed = _seed(opts)
    ctx = context(X.device)
    res = _lib.GmResult()
    with torch.cuda.device(X.device):
        _lib.check(ctx.lib.gm_weiszfeld_f32(ctx.handle, X.data_ptr(), K, d, ldx, g0.data_ptr(),
                                            out.data_ptr(), C.byref(o), C.byref(res),
                                            _stream_ptr(X.device)), "gm_weiszfeld_f32")
    last_result = _result(res)
    if pre_var is not None and not isinstance(wList, ClientPanels) and X is not wList:
        # a strided view was packed into a copy: the fused pre-noise landed in the
        # copy, and OMA's contract is in place on wList (M:351-352, as OMA() copies back)
        wList.copy_(X)
    return out if wList.device == out.device else out.to(wList.device)


def gm2(wList, options={}):  # noqa: B006 - the reference's signature (M:162)
    """Ideal Weiszfeld geometric median (MNIST_Air_weight.py:162-184)."""
    return _weiszfeld(wList, options, aircomp=False)


def gm(wList, options={}):  # noqa: B006 - the reference's signature (M:131)
    """AirComp Weiszfeld geometric median (MNIST_Air_weight.py:131-160)."""
    return _weiszfeld(wList, options, aircomp=True)


def _coordinate(wList, fn_name, *extra):
    if isinstance(wList, ClientPanels):          # the *_panels_f32 kernels (same results)
        X, ldx, fn_name = wList.data, wList.panel_stride, fn_name.replace("_f32", "_panels_f32")
        K, d = wList.shape
        out = torch.empty(d, dtype=torch.float32, device=X.device)
        ctx = context(X.device)
        with torch.cuda.device(X.device):
            _lib.check(getattr(ctx.lib, fn_name)(ctx.handle, X.data_ptr(), K, d, ldx, *extra,
                                                 out.data_ptr(), _stream_ptr(X.device)), fn_name)
        return out
    X = _stage(wList)
    X, ldx = _rows(X)
    K, d = X.shape
    out = torch.empty(d, dtype=torch.float32, device=X.device)
    ctx = context(X.device)
    with torch.cuda.device(X.device):
        _lib.check(getattr(ctx.lib, fn_name)(ctx.handle, X.data_ptr(), K, d, ldx, *extra,
                                             out.data_ptr(), _stream_ptr(X.device)), fn_name)
    return out if wList.device == out.device else out.to(wList.device)


def mean(wList, options={}):  # noqa: B006 - reference signature (M:186)
    """Column mean (MNIST_Air_weight.py:186-187)."""
    return _coordinate(wList, "gm_mean_f32")


def median(wList, options={}):  # noqa: B006 - reference signature (M:194)
    """Coordinate-wise lower median, torch.median semantics (M:194-195)."""
    return _coordinate(wList, "gm_median_f32")


def trimmed_mean(wList, options={}):  # noqa: B006 - reference signature (M:189)
    """Coordinate-wise mean without the int(0.1 K) smallest and largest (M:189-192)."""
    return _coordinate(wList, "gm_trimmed_mean_f32", int(wList.shape[0] * 0.1))


def Krum(wList, options):  # noqa: N802 - reference name (M:197)
    """The row with the smallest sum of squared distances to its honestSize-1
    nearest rows, itself included (M:197-204)."""
    if isinstance(wList, ClientPanels):
        X, ldx, fn = wList.data, wList.panel_stride, "gm_krum_panels_f32"
        K, d = wList.shape
    else:
        X = _stage(wList)
        X, ldx = _rows(X)
        K, d = X.shape
        fn = "gm_krum_f32"
    out = torch.empty(d, dtype=torch.float32, device=X.device)
    idx = C.c_int64()
    ctx = context(X.device)
    with torch.cuda.device(X.device):
        _lib.check(getattr(ctx.lib, fn)(ctx.handle, X.data_ptr(), K, d, ldx,
                                        int(options["honestSize"]), out.data_ptr(), C.byref(idx),
                                        _stream_ptr(X.device)), fn)
    info = (C.c_int64 * 3)()
    _lib.check(ctx.lib.gm_krum_last_info(ctx.handle, info), "gm_krum_last_info")
    Krum.last_index = idx.value
    Krum.last_info = {"algo": ("exact", "gram")[info[0]], "candidates": info[1],
                      "reason": ("ok", "not_chosen", "not_eligible", "gram_nonfinite",
                                 "candidates")[info[2]]}
    return out if wList.device == out.device else out.to(wList.device)


def honest_variance(w_local, honestSize: int) -> torch.Tensor:
    """getVarience (M:127-129) on the device: the mean over the first honestSize rows
    of ||x_k - mean||^2, one streaming pass (fp64 sums); a 0-dim fp32 tensor."""
    out = torch.empty((), dtype=torch.float32, device=w_local.device)
    if isinstance(w_local, ClientPanels):
        ctx = context(w_local.device)
        with torch.cuda.device(w_local.device):
            _lib.check(ctx.lib.gm_honest_variance_panels_f32(
                ctx.handle, w_local.data.data_ptr(), w_local.K, int(honestSize), w_local.d,
                w_local.panel_stride, out.data_ptr(), _stream_ptr(w_local.device)),
                "gm_honest_variance_panels_f32")
        return out
    if w_local.device.type != "cuda" or w_local.dtype != torch.float32 or w_local.dim() != 2:
        raise TypeError("honest_variance needs an fp32 CUDA [K, d] matrix or ClientPanels")
    X = w_local if (w_local.stride(1) == 1 and w_local.stride(0) >= w_local.shape[1]) \
        else w_local.contiguous()
    if not 1 <= honestSize <= X.shape[0]:
        raise ValueError(f"honestSize {honestSize} not in [1, {X.shape[0]}]")
    ctx = context(X.device)
    with torch.cuda.device(X.device):
        _lib.check(ctx.lib.gm_honest_variance_f32(
            ctx.handle, X.data_ptr(), int(honestSize), X.shape[1], max(X.stride(0), X.shape[1]),
            out.data_ptr(), _stream_ptr(X.device)), "gm_honest_variance_f32")
    return out


def OMA(message, noise_var=0.01, noise_source=None, seed=None):  # noqa: N802 - reference name
    """In-place per-client equalised AWGN (MNIST_Air_weight.py:385-394)."""
    if isinstance(message, ClientPanels):
        src = _noise_source({} if noise_source is None else {"noise_source": noise_source})
        if src == _lib.GM_NOISE_HOST:          # the reference's [K, d] draws: via rows
            rows = message.to_rows()
            OMA(rows, noise_var, noise_source=noise_source, seed=seed)
            message.copy_rows_(rows)
            return message
        ctx = context(message.device)
        with torch.cuda.device(message.device):
            _lib.check(ctx.lib.gm_oma_philox_panels_f32(
                ctx.handle, message.data.data_ptr(), message.K, message.d, message.panel_stride,
                float(noise_var), _seed({"seed": seed}), _stream_ptr(message.device)),
                "gm_oma_philox_panels_f32")
        return message
    if message.dtype != torch.float32:
        raise TypeError(f"OMA kernel is fp32 (got {message.dtype})")
    X = _stage(message)
    Xc = X if (X.stride(1) == 1 and X.stride(0) >= X.shape[1]) else X.contiguous()
    K, d = Xc.shape
    ldx = max(Xc.stride(0), d)
    ctx = context(Xc.device)
    src = _noise_source({} if noise_source is None else {"noise_source": noise_source})
    stream = _stream_ptr(Xc.device)
    with torch.cuda.device(Xc.device):
        if src == _lib.GM_NOISE_HOST:
            sd = math.sqrt(noise_var)
            hr = torch.normal(torch.zeros(K, 1), 1 / math.sqrt(2))     # M:389-392 order
            hi = torch.normal(torch.zeros(K, 1), 1 / math.sqrt(2))
            nr = torch.normal(torch.zeros(K, d), sd)
            ni = torch.normal(torch.zeros(K, d), sd)
            dev = [t.to(Xc.device) for t in (hr, hi, nr, ni)]
            _lib.check(ctx.lib.gm_oma_apply_f32(ctx.handle, Xc.data_ptr(), K, d, ldx,
                                                *[t.data_ptr() for t in dev], stream),
                       "gm_oma_apply_f32")
        else:
            s = _seed({"seed": seed})
            _lib.check(ctx.lib.gm_oma_philox_f32(ctx.handle, Xc.data_ptr(), K, d, ldx,
                                                 float(noise_var), s, stream),
                       "gm_oma_philox_f32")
    if Xc is not message:
        message.copy_(Xc)
    return message
