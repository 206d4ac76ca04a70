"""Client updates in the panel layout (GM_LAYOUT_PANELS, include/gmagg.h).

The reference hands its aggregator a fresh ``torch.stack`` of flattened client
vectors, row-major ``[K, d]`` (MNIST_Air_weight.py:206-209, M:353).  The
streaming Weiszfeld pass reads that matrix in chunks of W columns x all K rows
(DESIGN.md §3.1); in row-major order each chunk is K separate W*4-byte
segments, 4*d bytes apart.  ``ClientPanels`` stores the same K x d values as
``[ceil(d/W)][K][W]`` (W = ``gm_panel_width(K)``, 32 at 512 < K <= 1024), so
each chunk is ONE contiguous block of HBM.  It is the device-resident buffer a
training loop writes client rows into (``store``), and ``gm2`` / ``gm`` accept it
wherever they accept a ``[K, d]`` tensor; results are bit-identical to the
row-major call (same chunks, same reduction order).
"""
from __future__ import annotations

import torch

from . import _lib

__all__ = ["ClientPanels", "panel_width"]


def panel_width(K: int) -> int:
    """W of the panel layout for K clients (the streaming tile's chunk width)."""
    w = int(_lib.load().gm_panel_width(int(K)))
    if w <= 0:
        raise ValueError(f"no panel layout for K={K}")
    return w


class ClientPanels:
    """K client vectors of length d, stored as ``data[ceil(d/W), K, W]`` fp32."""

    def __init__(self, K: int, d: int, device=None, W: int | None = None):
        self.K, self.d = int(K), int(d)
        self.W = int(W) if W is not None else panel_width(K)
        self.npan = -(-self.d // self.W)
        dev = torch.device(device) if device is not None else torch.device("cuda")
        # zero-filled: the last panel's columns >= d stay 0
        self.data = torch.zeros(self.npan, self.K, self.W, dtype=torch.float32, device=dev)

    # -- shape / metadata, so callers can treat it like the [K, d] matrix --------
    @property
    def shape(self):
        return torch.Size((self.K, self.d))

    @property
    def device(self):
        return self.data.device

    @property
    def dtype(self):
        return self.data.dtype

    @property
    def panel_stride(self) -> int:
        return self.K * self.W

    def _full(self) -> int:
        return self.d // self.W

    # -- writing and reading rows ------------------------------------------------
    def store(self, k: int, vec: torch.Tensor):
        """Write client k's flattened vector (d floats) into its slots."""
        vec = vec.reshape(-1)
        if vec.numel() != self.d:
            raise ValueError(f"vector has {vec.numel()} elements, expected {self.d}")
        nf = self._full()
        with torch.no_grad():
            if nf:
                self.data[:nf, k, :].copy_(vec[:nf * self.W].view(nf, self.W))
            rem = self.d - nf * self.W
            if rem:
                self.data[nf, k, :rem].copy_(vec[nf * self.W:])

    def copy_rows_(self, X: torch.Tensor):
        """Fill from a row-major [K, d] matrix (any device; copied to ours)."""
        if tuple(X.shape) != (self.K, self.d):
            raise ValueError(f"rows must be [{self.K}, {self.d}] (got {tuple(X.shape)})")
        X = X.to(self.device)
        if X.device.type == "cuda" and X.dtype == torch.float32:
            # one HIP kernel (pack.hip, gm_rows_to_panels_f32) instead of torch's
            # transposed copy
            from . import _lib
            from .aggregators import context, _stream_ptr
            if X.stride(1) != 1 or X.stride(0) < self.d:
                X = X.contiguous()
            ctx = context(X.device)
            with torch.cuda.device(X.device):
                _lib.check(ctx.lib.gm_rows_to_panels_f32(
                    ctx.handle, X.data_ptr(), self.K, self.d, max(X.stride(0), self.d),
                    self.data.data_ptr(), self.W, self.panel_stride, _stream_ptr(X.device)),
                    "gm_rows_to_panels_f32")
            return self
        nf = self._full()
        with torch.no_grad():
            if nf:
                self.data[:nf].copy_(X[:, :nf * self.W].view(self.K, nf, self.W).transpose(0, 1))
            rem = self.d - nf * self.W
            if rem:
                self.data[nf, :, :rem].copy_(X[:, nf * self.W:])
        return self

    @classmethod
    def from_rows(cls, X: torch.Tensor, device=None) -> "ClientPanels":
        K, d = X.shape
        p = cls(K, d, device=device if device is not None else
                (X.device if X.device.type == "cuda" else None))
        return p.copy_rows_(X)

    def row(self, k: int) -> torch.Tensor:
        return self.data[:, k, :].reshape(-1)[: self.d]

    def to_rows(self) -> torch.Tensor:
        """The row-major [K, d] matrix (a copy)."""
        return self.data.transpose(0, 1).reshape(self.K, self.npan * self.W)[:, : self.d].contiguous()

    def mean(self, dim: int = 0) -> torch.Tensor:
        """Column mean (gm2's default guess, M:167)."""
        if dim != 0:
            raise ValueError("ClientPanels.mean supports dim=0 only")
        return self.data.mean(dim=1).reshape(-1)[: self.d]
