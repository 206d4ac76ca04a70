"""Many independent aggregations in one launch per pass (BASELINE C5).

The reference's results figure (draw.ipynb) is a sweep over aggregator x noise
variance x Byzantine count, each point being thousands of `gm2`/`gm` calls.
Here P problems [P, K, d] run together: every streaming pass covers all of
them (grid = chunk blocks x problems), each problem keeps its own K-space
state and stops at its own tol test (gm2) or runs to maxiter (gm, which never
meets tol).  AirComp problems draw from Philox, problem p keyed with
seed + p * 0x9E3779B97F4A7C15, so problem p equals a single `gm` call with that
seed.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .aggregators import GMResult, _ALGOS, _result, _seed, _stream_ptr, context
from .panels import panel_width

__all__ = ["gm2_batched", "gm_batched", "oma_batched", "ProblemPanels", "SEED_STRIDE"]

SEED_STRIDE = 0x9E3779B97F4A7C15


class ProblemPanels:
    """P independent client matrices (K x d each) in the panel layout: ``data[P, npan, K, W]``
    (W = ``panel_width(K)``), each problem a ``ClientPanels``-layout block, so that every
    streaming chunk of every problem is one contiguous block of HBM.  The batched calls
    accept it in place of a ``[P, K, d]`` tensor; results are bit-identical to the
    row-major batched call where both run the same tile (K outside 32 < K <= 64 and
    128 < K <= 256, d % 4 == 0), equal to rounding otherwise."""

    def __init__(self, P: int, K: int, d: int, device=None):
        self.P, self.K, self.d = int(P), int(K), int(d)
        self.W = panel_width(self.K)
        self.npan = -(-self.d // self.W)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        self.data = torch.zeros(self.P, self.npan, self.K, self.W, dtype=torch.float32, device=dev)

    @property
    def shape(self):
        return torch.Size((self.P, self.K, self.d))

    @property
    def device(self):
        return self.data.device

    @property
    def panel_stride(self) -> int:
        return self.K * self.W

    @property
    def problem_stride(self) -> int:
        return self.npan * self.K * self.W

    def copy_rows_(self, X: torch.Tensor):
        """Fill from row-major problems X [P, K, d] (on the device: one pack kernel each)."""
        if tuple(X.shape) != (self.P, self.K, self.d):
            raise ValueError(f"rows must be [{self.P}, {self.K}, {self.d}] (got {tuple(X.shape)})")
        X = X.to(self.device, torch.float32)
        if X.stride(2) != 1:
            X = X.contiguous()
        ctx = context(self.device)
        with torch.cuda.device(self.device):
            for p in range(self.P):
                _lib.check(ctx.lib.gm_rows_to_panels_f32(
                    ctx.handle, X[p].data_ptr(), self.K, self.d, X.stride(1),
                    self.data[p].data_ptr(), self.W, self.panel_stride,
                    _stream_ptr(self.device)), "gm_rows_to_panels_f32")
        return self

    @classmethod
    def from_rows(cls, X: torch.Tensor):
        P, K, d = X.shape
        return cls(P, K, d, device=X.device).copy_rows_(X)

    def to_rows(self) -> torch.Tensor:
        full = self.data.permute(0, 2, 1, 3).reshape(self.P, self.K, self.npan * self.W)
        return full[:, :, :self.d].contiguous()


def _run(X, options: dict, aircomp: bool):
    X_in = X
    panels = isinstance(X, ProblemPanels)
    if panels:
        P, K, d = X.shape
        buf, ldx, ldp = X.data, X.panel_stride, X.problem_stride
    else:
        if X.dim() != 3:
            raise ValueError(f"X must be [P, K, d] (got {tuple(X.shape)})")
        if X.device.type != "cuda" or X.dtype != torch.float32:
            raise TypeError("batched aggregation needs an fp32 CUDA tensor")
        if X.stride(2) != 1 or X.stride(1) < X.shape[2] or X.stride(0) < X.shape[1] * X.stride(1):
            X = X.contiguous()
        P, K, d = X.shape
        buf, ldx, ldp = X, X.stride(1), X.stride(0)
    opts = {"maxiter": 200, "tol": 1e-5, "noise_var": None, "P_max": 1}
    opts.update(options or {})
    # pre_oma_var (gm2): the `--agg gm2 --var v` pre-noise (M:351-352) in place, fused
    # into the INIT pass; problem p keyed pre_oma_seed + p * SEED_STRIDE as oma_batched.
    # The default guess is the mean of the NOISY rows: then the separate OMA runs first.
    pre_var = None if aircomp else opts.get("pre_oma_var")
    pre_seed = int(opts.get("pre_oma_seed", 2021)) & 0xFFFFFFFFFFFFFFFF
    if pre_var is not None and opts.get("guess") is None:
        oma_batched(X, float(pre_var), seed=pre_seed)
        if X is not X_in:
            X_in.copy_(X)      # OMA is in place on the caller's problems (M:351-352)
        pre_var = None
    guess = opts.get("guess")
    if guess is None:
        guess = (X.to_rows() if panels else X).mean(dim=1)
    g0 = guess.to(device=X.device, dtype=torch.float32).contiguous()
    if tuple(g0.shape) != (P, d):
        raise ValueError(f"guess must be [P, d] = [{P}, {d}]")
    out = torch.empty(P, d, dtype=torch.float32, device=X.device)
    o = _lib.GmOpts()
    o.maxiter = int(opts["maxiter"])
    o.tol = float(opts["tol"])
    o.eps = 1e-4
    o.mode = _lib.GM_MODE_AIRCOMP if aircomp else _lib.GM_MODE_IDEAL
    o.check_every = int(opts.get("check_every", 0))
    o.layout = _lib.GM_LAYOUT_PANELS if panels else _lib.GM_LAYOUT_ROWS
    # "auto" (problems that fit on chip run register-resident, X read once), "stream"
    # (one streaming pass per iteration over every problem) or "resident" (raises if the
    # shape does not fit)
    o.algo = _ALGOS[opts.get("algo", "auto")]
    if pre_var is not None:
        o.pre_oma = 1
        o.pre_oma_var = float(pre_var)
        o.pre_oma_seed = pre_seed
    if aircomp:
        var = opts["noise_var"]
        o.has_noise = int(var is not None)
        o.noise_var = float(var) if var is not None else 0.0
        o.P_max = float(opts["P_max"])
        o.seed = _seed(opts)
    res = (_lib.GmResult * P)()
    ctx = context(X.device)
    with torch.cuda.device(X.device):
        _lib.check(ctx.lib.gm_weiszfeld_batched_f32(
            ctx.handle, buf.data_ptr(), P, K, d, ldx, ldp, g0.data_ptr(), d,
            out.data_ptr(), d, C.byref(o), res, _stream_ptr(X.device)), "gm_weiszfeld_batched_f32")
    if pre_var is not None and X is not X_in:
        X_in.copy_(X)          # the fused pre-noise is in place on the caller's problems
    results = [_result(r) for r in res]
    return out, results


def oma_batched(X, noise_var: float, seed: int = 2021):
    """OMA pre-noise (M:385-394) in place on each of P problems X[p] ([P, K, d] or
    ProblemPanels): the reference's `--agg gm2 --var v` path adds it before gm2
    (M:351-352).  Problem p's draws equal `aggregators.OMA(X[p], noise_var, seed + p *
    SEED_STRIDE)`, in either layout."""
    if isinstance(X, ProblemPanels):
        ctx = context(X.device)
        with torch.cuda.device(X.device):
            _lib.check(ctx.lib.gm_oma_philox_batched_panels_f32(
                ctx.handle, X.data.data_ptr(), X.P, X.K, X.d, X.panel_stride, X.problem_stride,
                float(noise_var), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream_ptr(X.device)),
                "gm_oma_philox_batched_panels_f32")
        return X
    if X.dim() != 3 or X.device.type != "cuda" or X.dtype != torch.float32 or X.stride(2) != 1:
        raise TypeError("oma_batched needs an fp32 CUDA [P, K, d] tensor with unit column stride")
    P, K, d = X.shape
    ctx = context(X.device)
    with torch.cuda.device(X.device):
        _lib.check(ctx.lib.gm_oma_philox_batched_f32(
            ctx.handle, X.data_ptr(), P, K, d, X.stride(1), X.stride(0), float(noise_var),
            int(seed) & 0xFFFFFFFFFFFFFFFF, _stream_ptr(X.device)), "gm_oma_philox_batched_f32")
    return X


def gm2_batched(X, options=None):
    """gm2 (M:162-184) on each of P problems X[p] ([P, K, d]) -> ([P, d], results)."""
    return _run(X, options or {}, aircomp=False)


def gm_batched(X, options=None):
    """AirComp gm (M:131-160) on each of P problems, Philox noise -> ([P, d], results)."""
    return _run(X, options or {}, aircomp=True)
