"""Op-for-op PyTorch-CPU restatement of the reference's aggregation path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the checker for the HIP
path and the timed ``cpu_baseline`` of ``bench.py``.  Never shipped, never
called by ``byzantine_aircomp_amd``.

Reference = goldenBill/Byzantine_AirComp, ``MNIST_Air_weight.py`` (cited "M:")
— ``EMNIST_Air_weight.py`` holds the same functions at the same lines
131-204 and ``OMA``/``OMA2`` at +2 lines.

Every function keeps the reference's fp32 temporaries and op order, so on the
same inputs and the same CPU-generator state it reproduces the reference to the
last bit (pinned by ``tests/test_oracle_golden.py`` against fixtures made by
importing the reference).  In addition to the aggregate, the Weiszfeld
restatements report what the reference computes but does not return: the
number of loop bodies executed and the last ``guess_movement``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Callable, Optional

import torch

CLAMP = 1e-4  # M:151 / M:178 distance floor


@dataclass
class WeiszfeldTrace:
    """What a Weiszfeld run did, beyond its return value."""

    iters: int            # loop bodies executed (M:145 / M:173)
    last_movement: float  # ||guess_t - guess_{t+1}|| of the final body, nan if none


def _with_defaults(wList: torch.Tensor, options: dict, defaults: dict) -> dict:
    # M:136-138 / M:167-169: the defaults dict is built EAGERLY, so the mean
    # (K x d pass) is computed even when a guess is supplied.
    merged = dict(defaults)
    merged["guess"] = wList.mean(dim=0)
    merged.update(options)
    return merged


def _clamped_row_distances(wList: torch.Tensor, guess: torch.Tensor) -> torch.Tensor:
    # M:174 + M:178 (same as M:147 + M:151): fp32 row norms, floor 1e-4 held in
    # an fp32 0-d tensor and applied with torch.max (NaN propagates).
    dist = torch.norm(wList - guess, dim=1)
    return torch.max(torch.tensor(CLAMP).to(wList.device), dist)


def gm2(wList: torch.Tensor, options: Optional[dict] = None):
    """Ideal Weiszfeld geometric median, M:162-184.  Returns (guess, trace)."""
    opts = _with_defaults(wList, options or {}, {"maxiter": 200, "tol": 1e-5})
    guess = opts["guess"]
    n, moved = 0, float("nan")
    for _ in range(opts["maxiter"]):
        n += 1
        dist = _clamped_row_distances(wList, guess)
        nxt = (wList / dist.unsqueeze(-1)).sum(dim=0) / (1 / dist).sum()   # M:179
        movement = (guess - nxt).norm()                                    # M:180
        moved = float(movement)
        guess = nxt                                                         # M:181
        if movement <= opts["tol"]:                                        # M:182
            break
    return guess, WeiszfeldTrace(n, moved)


def oma2(message: torch.Tensor, P_max=10, noise_var=None, threshold=1,
         draw: Optional[Callable] = None) -> torch.Tensor:
    """AirComp weighted sum with truncated channel inversion, M:396-414.

    ``draw(shape, std)`` supplies the normals; default is the reference's own
    ``torch.normal(torch.zeros(shape), std)`` on the global CPU generator, in
    the reference's order: channel real [K], channel imag [K], noise [d+1].
    """
    draw = draw or (lambda shape, std: torch.normal(torch.zeros(*shape), std))
    msg = message.clone().detach()
    K, L = msg.shape
    h_re = draw((K,), 1 / math.sqrt(2)).to(message.device)
    h_im = draw((K,), 1 / math.sqrt(2)).to(message.device)
    h2 = h_re ** 2 + h_im ** 2                                  # M:403
    p_up = torch.max(torch.mean(msg ** 2 / h2.unsqueeze(-1), dim=-1), threshold)  # M:404-405
    gain = torch.sqrt(P_max / p_up)                              # M:407
    summed = (msg * gain.unsqueeze(-1)).sum(dim=0)               # M:408
    if noise_var is None:
        return summed                                            # M:414
    noise = draw((L,), math.sqrt(noise_var / 2)).to(message.device)
    return summed.add_(noise)                                    # M:409-412


def gm(wList: torch.Tensor, options: Optional[dict] = None,
       draw: Optional[Callable] = None):
    """AirComp Weiszfeld geometric median, M:131-160.  Returns (guess, trace)."""
    opts = _with_defaults(wList, options or {},
                          {"maxiter": 200, "tol": 1e-5, "noise_var": None, "P_max": 1})
    guess = opts["guess"]
    n, moved = 0, float("nan")
    for _ in range(opts["maxiter"]):
        n += 1
        scaler = torch.sqrt(torch.mean(guess ** 2))               # M:146
        dist = _clamped_row_distances(wList, guess)               # M:147, M:151
        msg = torch.cat([wList / dist.unsqueeze(-1), scaler / dist.unsqueeze(-1)], dim=-1)
        y = oma2(msg, P_max=opts["P_max"], noise_var=opts["noise_var"],
                 threshold=(scaler ** 2) * 500, draw=draw)        # M:152
        nxt = y[:-1] / y[-1:] * scaler                            # M:153-155
        movement = (guess - nxt).norm()                           # M:156
        moved = float(movement)
        guess = nxt
        if movement <= opts["tol"]:                               # M:158
            break
    return guess, WeiszfeldTrace(n, moved)


def oma_(message: torch.Tensor, noise_var: float = 0.01, draw: Optional[Callable] = None):
    """Per-client equalised AWGN, applied in place, M:385-394.

    Draw order (M:389-392): channel real [K,1], channel imag [K,1], noise
    real [K,d], noise imag [K,d]; std 1/sqrt(2) for the channel and
    sqrt(noise_var) for the noise.
    """
    draw = draw or (lambda shape, std: torch.normal(torch.zeros(*shape), std))
    K, d = message.shape
    sd = math.sqrt(noise_var)
    h_re = draw((K, 1), 1 / math.sqrt(2)).to(message.device)
    h_im = draw((K, 1), 1 / math.sqrt(2)).to(message.device)
    n_re = draw((K, d), sd).to(message.device)
    n_im = draw((K, d), sd).to(message.device)
    message[:].add_((h_re * n_re + h_im * n_im) / (h_re ** 2 + h_im ** 2))   # M:393-394
    return message


# --- alternative aggregators, M:186-204 -------------------

def mean(wList, options=None):
    return torch.mean(wList, dim=0)                               # M:186-187


def trimmed_mean(wList, options=None):
    K = wList.shape[0]
    b = int(K * 0.1)                                              # M:191
    low = wList.topk(K - b, dim=0, largest=False)[0]
    return torch.mean(low.topk(K - 2 * b, dim=0, largest=True)[0], dim=0)   # M:192


def median(wList, options=None):
    return wList.median(dim=0)[0]                                 # M:194-195 (lower median)


def krum(wList, options):
    honest = options["honestSize"]
    d2 = ((wList.unsqueeze(1) - wList.unsqueeze(0)) ** 2).sum(dim=-1)   # M:199
    score = d2.topk(k=honest - 1, dim=1, largest=False)[0].sum(dim=1)  # M:200-202
    return wList[score.argmin()]                                  # M:203-204


def variance(wList, honest):
    """getVarience, M:127-129."""
    h = wList[:honest]
    return torch.mean(((h - h.mean(dim=0)) ** 2).sum(dim=1))


# --- fp64 K-space cross-check (not op-for-op; used to bound fp32 drift) ------

def gm2_f64(X: torch.Tensor, guess: torch.Tensor, maxiter: int = 200, tol: float = 1e-5):
    """Weiszfeld in float64 on the same inputs; returns (guess_f64, trace)."""
    X64, g = X.double(), guess.double()
    n, moved = 0, float("nan")
    for _ in range(maxiter):
        n += 1
        dist = torch.clamp(torch.linalg.vector_norm(X64 - g, dim=1), min=CLAMP)
        w = 1.0 / dist
        nxt = (w @ X64) / w.sum()
        moved = float(torch.linalg.vector_norm(g - nxt))
        g = nxt
        if moved <= tol:
            break
    return g, WeiszfeldTrace(n, moved)


# The fp32 movement floor, in ulps of ||g||: an fp32 Weiszfeld's computed movement differs
# from the exact one by about this much (profiles/r5s1_movement_floor.txt: <= 2.0 ulps at the
# tol crossing on every C4-recipe input, 0.6-1.0 ulps at the fixed point).  The SAME constant
# as the Gram guard's floor rule (byzantine_aircomp_amd/csrc/gmagg_internal.h kFloorUlps,
# api.hip run_gram; tests/test_iteration_wellposed.py checks the two agree).
FLOOR_ULPS = 2.0


@dataclass
class CountWindow:
    """The iteration counts an fp32 Weiszfeld may legitimately stop at on one input."""

    early: int            # first t whose fp64 movement is <= tol + delta_t
    late: Optional[int]   # first t whose fp64 movement is <= tol - delta_t (maxiter if none);
                          # None = undetermined: tol - delta <= 0, no count is certain
    max_norm: float       # max ||g_t|| over the run (sets the fp32 movement floor)

    @property
    def determined(self) -> bool:
        return self.late is not None

    @property
    def width(self) -> Optional[int]:
        return None if self.late is None else self.late - self.early


def gm2_count_window(X: torch.Tensor, guess: Optional[torch.Tensor] = None, maxiter: int = 200,
                     tol: float = 1e-5, floor_ulps: float = FLOOR_ULPS,
                     chunk_rows: Optional[int] = None) -> CountWindow:
    """Is "the same iteration count +-1" (north_star) well posed on this input?

    The reference stops at the first t with ||g_t - g_{t+1}|| <= tol (M:180-183), on
    fp32 iterates.  An fp32 iterate carries an error of a few ulps of its elements, so
    the movement an fp32 implementation computes differs from the exact one by up to
    delta_t ~ floor_ulps * 2^-24 * ||g_t|| (summation order decides the sign).  Any
    count between ``early`` (exact movement <= tol + delta) and ``late`` (exact
    movement <= tol - delta) is then a legitimate stopping point, for the reference as
    for a kernel: two fp32 implementations agree to +-1 only if ``late - early <= 1``.
    A wider window means tol sits near the fp32 movement floor and the count measures
    rounding, not the algorithm (6 vs 8 at ||g|| ~ 8, tol 1e-6).  When
    tol - delta <= 0 the window is UNDETERMINED (``late`` None): an fp32 run may never
    see a movement below tol (it stops only if rounding happens to land it there, or on
    an exact fixed point of its own arithmetic), so no count is certain and a test must
    state its own bar.  Runs the exact (fp64) iteration until the movement is below
    tol - delta.  ``chunk_rows``: convert and process X that many rows at a time (bounded
    fp64 temporaries for large inputs; the same iteration up to fp64 summation order)."""
    K = X.shape[0]
    step = K if chunk_rows is None else max(1, int(chunk_rows))
    X64 = X.double() if step >= K else None

    def rows(k0):
        return X64[k0:k0 + step] if X64 is not None else X[k0:k0 + step].double()

    g = (sum(rows(k0).sum(dim=0) for k0 in range(0, K, step)) / K if guess is None
         else guess.double())
    early = late = None
    undetermined = False
    max_norm = float(torch.linalg.vector_norm(g))
    for t in range(1, maxiter + 1):
        dist = torch.cat([torch.linalg.vector_norm(rows(k0) - g, dim=1)
                          for k0 in range(0, K, step)])
        dist = torch.clamp(dist, min=CLAMP)
        w = 1.0 / dist
        nxt = sum(w[k0:k0 + step] @ rows(k0) for k0 in range(0, K, step)) / w.sum()
        moved = float(torch.linalg.vector_norm(g - nxt))
        max_norm = max(max_norm, float(torch.linalg.vector_norm(nxt)))
        delta = floor_ulps * 2.0 ** -24 * max_norm
        g = nxt
        if early is None and moved <= tol + delta:
            early = t
        if moved <= tol - delta:
            late = t
            break
        if not math.isfinite(moved):
            break                   # NaN never passes the test: both run to maxiter
        if early is not None and tol - delta <= 0:
            undetermined = True     # (tol below the floor: no count is certain)
            break
    early = maxiter if early is None else early
    if undetermined:
        return CountWindow(early, None, max_norm)
    late = maxiter if late is None else late
    return CountWindow(early, late, max_norm)
