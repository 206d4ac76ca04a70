"""numpy restatement of the build's counter-based noise (byzantine_aircomp_amd/csrc/philox.h).

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``): the checker for the HIP
Philox paths, never called by ``byzantine_aircomp_amd``.

The reference draws its AirComp noise from torch's CPU generator (OMA M:385-394,
OMA2 M:401-411); the build's production path replaces those draws with
Philox4x32-10 (Salmon et al., SC'11) keyed by (seed, stream, iteration, index),
so any d-shard regenerates its own columns.  This module states that keying and
the Box-Muller transform in float64, so a GPU result can be checked draw by draw
(the device uses the hardware log2/sqrt/sin/cos: ~1 ulp of fp32 apart).
"""
from __future__ import annotations

import numpy as np

STREAM_OMA_CHANNEL = 0x4F4D4143
STREAM_OMA_NOISE = 0x4F4D414E
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, seed: int):
    """Philox4x32-10 on uint64 arrays holding 32-bit words (philox.h:30-41)."""
    c = [np.asarray(x, dtype=np.uint64) & MASK for x in (c0, c1, c2, c3)]
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK
        c = [hi1 ^ c[1] ^ np.uint64(k0), lo1, hi0 ^ c[3] ^ np.uint64(k1), lo0]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return c


def _u01(v):
    return ((v >> np.uint64(8)).astype(np.float64) + 1.0) / 16777216.0


def normal4(seed: int, stream: int, it, idx):
    """Four standard normals per (iteration, index) counter (philox.h normal4 / normal4_hw)."""
    it = np.asarray(it, dtype=np.uint64)
    idx = np.asarray(idx, dtype=np.uint64)
    r = philox4x32_10(idx & MASK, idx >> np.uint64(32), it & MASK,
                      np.uint64(stream) ^ (it >> np.uint64(32)), seed)
    out = []
    for a, b in ((r[0], r[1]), (r[2], r[3])):
        rad = np.sqrt(-2.0 * np.log(_u01(a)))
        t = 2.0 * np.pi * _u01(b)
        out += [rad * np.cos(t), rad * np.sin(t)]
    return np.stack(out, axis=-1)                   # [..., 4]


def oma_philox(X: np.ndarray, noise_var: float, seed: int, col_off: int = 0) -> np.ndarray:
    """X + the build's OMA noise (oma.hip oma_philox): client k's channel h_k is
    normals 0, 1 of block (iteration 0, index k) scaled by 1/sqrt(2); element
    (k, global column c) adds sqrt(var)/|h_k| times normal c & 3 of block
    (iteration k, index c >> 2)."""
    K, d = X.shape
    h = normal4(seed, STREAM_OMA_CHANNEL, np.zeros(K, dtype=np.uint64), np.arange(K))
    a, b = h[:, 0] / np.sqrt(2.0), h[:, 1] / np.sqrt(2.0)
    scale = np.sqrt(noise_var) / np.sqrt(a * a + b * b)
    cols = col_off + np.arange(d, dtype=np.uint64)
    z = normal4(seed, STREAM_OMA_NOISE, np.arange(K, dtype=np.uint64)[:, None],
                (cols >> np.uint64(2))[None, :])      # [K, d, 4]
    pick = np.take_along_axis(z, (cols & np.uint64(3)).astype(np.int64)[None, :, None]
                              .repeat(K, axis=0), axis=2)[..., 0]
    return X.astype(np.float64) + scale[:, None] * pick


STREAM_FILL = 0x46494C4C


_FILL_LIB = None


def _fill_lib():
    """oracle/_philox_fill.so (oracle/philox_fill.c, built by __graft_entry__.build() or on
    first use with gcc), or None: the numpy restatement below is then used."""
    global _FILL_LIB
    if _FILL_LIB is None:
        import ctypes
        import os
        import subprocess
        here = os.path.dirname(os.path.abspath(__file__))
        so, src = os.path.join(here, "_philox_fill.so"), os.path.join(here, "philox_fill.c")
        try:
            if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
                subprocess.run(["gcc", "-O2", "-fopenmp", "-shared", "-fPIC", src, "-o", so, "-lm"],
                               check=True, capture_output=True)
            lib = ctypes.CDLL(so)
            i64, u64, f64, fp = ctypes.c_int64, ctypes.c_uint64, ctypes.c_double, ctypes.c_void_p
            lib.fill_clients.argtypes = [i64, i64, i64, f64, f64, f64, f64, u64, i64, fp]
            lib.fill_normal.argtypes = [i64, f64, f64, u64, i64, fp]
            _FILL_LIB = lib
        except (OSError, subprocess.CalledProcessError):
            _FILL_LIB = False
    return _FILL_LIB or None


def fill_clients(K: int, d: int, B: int, mu_h: float, sd_h: float, mu_b: float, sd_b: float,
                 seed: int, col_off: int = 0) -> np.ndarray:
    """The synthetic client matrix of ``gm_fill_clients_f32`` (oma.hip fill_clients):
    element (k, global column c) = mu + sd * normal c & 3 of block (iteration k, index
    c >> 2) on the fill stream; the last B rows take (mu_b, sd_b).  float32 of the
    float64 Box-Muller: the device's fast sin/cos put it within ~1e-6 of this, enough
    to decide whether a test input is well posed (tests/test_iteration_wellposed.py)."""
    lib = _fill_lib()
    if lib is not None:
        X = np.empty((K, d), dtype=np.float32)
        lib.fill_clients(K, d, B, mu_h, sd_h, mu_b, sd_b, seed, col_off, X.ctypes.data)
        return X
    cols = col_off + np.arange(d, dtype=np.uint64)
    X = np.empty((K, d), dtype=np.float32)
    for k in range(K):
        z = normal4(seed, STREAM_FILL, np.uint64(k), cols >> np.uint64(2))     # [d, 4]
        v = np.take_along_axis(z, (cols & np.uint64(3)).astype(np.int64)[:, None], axis=1)[:, 0]
        mu, sd = (mu_b, sd_b) if k >= K - B else (mu_h, sd_h)
        X[k] = (mu + sd * v).astype(np.float32)
    return X


def fill_normal(n: int, mu: float, sd: float, seed: int, off: int = 0) -> np.ndarray:
    """``gm_fill_normal_f32`` (oma.hip fill_normal): normal c & 3 of block
    (iteration 0xFFFFFFFF, index c >> 2)."""
    lib = _fill_lib()
    if lib is not None:
        v = np.empty(n, dtype=np.float32)
        lib.fill_normal(n, mu, sd, seed, off, v.ctypes.data)
        return v
    cols = off + np.arange(n, dtype=np.uint64)
    z = normal4(seed, STREAM_FILL, np.uint64(0xFFFFFFFF), cols >> np.uint64(2))
    v = np.take_along_axis(z, (cols & np.uint64(3)).astype(np.int64)[:, None], axis=1)[:, 0]
    return (mu + sd * v).astype(np.float32)


STREAM_CHANNEL = 0x43484E4C
STREAM_NOISE = 0x4E4F4953


def gm_draws(seed: int, d_total: int, col_off: int = 0):
    """A ``draw(shape, std)`` for ``oracle.aggregators.gm`` that supplies the build's
    Philox AirComp draws in the reference's per-iteration order (OMA2 M:401-402,
    M:411: channel real [K], channel imag [K], noise [d+1]).  Iteration it's client
    k takes normals 0 / 1 of block (it, k) on the channel stream (weiszfeld.hip
    kspace_step); global column j's noise is normal j & 3 of block (it, j >> 2) on the
    noise stream, the denominator's entry is global index d_total (philox.h normal1)."""
    import torch
    state = {"it": 0, "call": 0, "h": None}

    def draw(shape, std):
        it, call = state["it"], state["call"]
        if call == 0:
            n = shape[0]
            state["h"] = normal4(seed, STREAM_CHANNEL, np.uint64(it), np.arange(n, dtype=np.uint64))
            v = state["h"][:, 0]
        elif call == 1:
            v = state["h"][:, 1]
        else:
            L = shape[0]                                  # d + 1
            idx = np.concatenate([col_off + np.arange(L - 1, dtype=np.uint64),
                                  np.array([d_total], dtype=np.uint64)])
            z = normal4(seed, STREAM_NOISE, np.uint64(it), idx >> np.uint64(2))     # [L, 4]
            v = np.take_along_axis(z, (idx & np.uint64(3)).astype(np.int64)[:, None], axis=1)[:, 0]
        state["call"] = call + 1
        if call == 2 or (call == 1 and state.get("no_noise")):
            state["it"], state["call"] = it + 1, 0
        return torch.from_numpy((v * std).astype(np.float32))

    def no_noise():
        state["no_noise"] = True

    draw.no_noise = no_noise
    return draw
