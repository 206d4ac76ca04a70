"""d-sharded geometric median across GPUs (one process per GPU).

The reference runs its aggregator in one process on CPU tensors; at the
C3/C4 sizes (K x d = 1000 x 11M, 256 x 125M) the build shards the d axis:
rank r holds the contiguous column range ``shard_range(d, world, r)`` of
every client row and of the iterate.  Each Weiszfeld iteration needs exactly
one exchange — an all-reduce (sum) of the (K+2)-vector of fp64 partials
[per-row squared distances | movement^2 | ||g||^2] — after which every rank
derives identical weights and takes the identical stop decision.  The
aggregate stays shard-local.  AirComp channel draws and column noise are
counter-based Philox keyed by (seed, iteration, GLOBAL index), so the ranks
agree without communicating.

The all-reduce is RCCL over xGMI, called natively by libgmagg (the rank-0
ncclUniqueId is shared through the caller's torch.distributed group), or —
``transport="torch"`` — any torch.distributed backend through the library's
all-reduce callback (used by the CPU/gloo tests of the host logic).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib
from .aggregators import GMResult, Context, _ALGOS, _noise_source, _result, _seed
from .panels import ClientPanels

__all__ = ["shard_range", "ShardedGM", "torch_allreduce_adapter"]

ALIGN = 256   # columns; keeps every shard's rows 1 KiB-aligned for the float4 tiles


def shard_range(d: int, world: int, rank: int, align: int = ALIGN):
    """[lo, hi) columns of rank `rank`: equal `align`-rounded slices, the tail ragged."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"rank {rank} of {world}")
    per = -(-d // world)
    per = -(-per // align) * align
    lo = min(d, rank * per)
    return lo, min(d, lo + per)


def _wrap(ptr: int, count: int, device: torch.device) -> torch.Tensor:
    """A torch view of `count` doubles at raw address `ptr` (no copy)."""
    if device.type == "cpu":
        buf = (C.c_double * count).from_address(ptr)
        return torch.frombuffer(buf, dtype=torch.float64, count=count)

    class _Iface:
        __cuda_array_interface__ = {"shape": (count,), "typestr": "<f8", "data": (ptr, False),
                                    "version": 2, "strides": None}
    return torch.as_tensor(_Iface(), device=device)


def torch_allreduce_adapter(group=None, device: torch.device | None = None):
    """fn(ptr, count, stream) summing doubles in place with torch.distributed."""
    import torch.distributed as dist

    def fn(ptr, count, stream):
        dev = device or torch.device("cpu")
        t = _wrap(ptr, count, dev)
        if dev.type == "cuda":
            s = torch.cuda.ExternalStream(stream, device=dev) if stream else torch.cuda.current_stream(dev)
            with torch.cuda.stream(s):
                dist.all_reduce(t, group=group)
        else:
            dist.all_reduce(t, group=group)
    return fn


def _aligned(shards, d_total: int) -> bool:
    """Every rank's shard lies in [0, d_total), 256-aligned at lo and 4-aligned at hi
    (so d_total % 4 == 0 gives every rank the float4 rows the Gram path needs).  With
    more than one rank the shards must also tile [0, d_total) — contiguous, no overlap,
    no gap — or the all-reduced distances sum over the wrong set of columns; a single
    rank may hold any shard (a one-GPU rehearsal of rank r of a larger job)."""
    if not all(0 <= lo <= hi <= d_total and lo % ALIGN == 0 and (hi % 4 == 0 or hi == d_total)
               for lo, hi in shards):
        return False
    if len(shards) == 1:
        return True
    end = 0
    for lo, hi in sorted(shards):
        if lo != end:
            return False
        end = hi
    return end == d_total


class ShardedGM:
    """gm2 / gm on this rank's column shard of a d_total-long update."""

    def __init__(self, d_total: int, group=None, device: torch.device | None = None,
                 transport: str = "rccl", shard: tuple[int, int] | None = None):
        """``shard`` overrides this rank's [lo, hi) columns (default: the even
        ``shard_range`` plan).  Every rank's shard must then start at a multiple of
        256 columns and the shards must tile [0, d_total) — a one-GPU rehearsal of
        rank r of a larger job passes ``shard_range(d_total, P, r)`` at world size 1."""
        import torch.distributed as dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.d_total = d_total
        if shard is None:
            self.lo, self.hi = shard_range(d_total, self.world, self.rank)
        else:
            self.lo, self.hi = int(shard[0]), int(shard[1])
            # validated collectively: a shard that only one rank rejects (or that only one
            # rank's library call would refuse inside a collective sequence) hangs the rest
            shards = [None] * self.world
            dist.all_gather_object(shards, (self.lo, self.hi), group=group)
            if not _aligned(shards, d_total):
                raise ValueError(f"shards {shards} of d_total={d_total}: each must be [lo, hi) "
                                 f"within [0, d_total) with lo % {ALIGN} == 0 and hi % 4 == 0 "
                                 "(or hi == d_total), tiling [0, d_total) at world size > 1")
        self.ctx = Context(self.device.index)
        self.ctx.set_shard(d_total, self.lo)
        if transport == "rccl":
            uid = [None]
            if self.rank == 0:
                buf = C.create_string_buffer(128)
                _lib.check(self.ctx.lib.gm_rccl_get_unique_id(buf), "gm_rccl_get_unique_id")
                uid[0] = buf.raw
            dist.broadcast_object_list(uid, src=dist.get_global_rank(group, 0) if group else 0,
                                       group=group)
            self.ctx.init_rccl(uid[0], self.world, self.rank)
        elif transport == "torch":
            self.ctx.set_allreduce(torch_allreduce_adapter(group, self.device))
        else:
            raise ValueError(f"transport must be 'rccl' or 'torch' (got {transport!r})")
        self.last_result: GMResult | None = None

    @property
    def d_local(self) -> int:
        return self.hi - self.lo

    def _run(self, X: torch.Tensor, options: dict, aircomp: bool) -> torch.Tensor:
        opts = {"maxiter": 200, "tol": 1e-5, "noise_var": None, "P_max": 1}
        opts.update(options or {})
        if X.shape[1] != self.d_local or X.device != self.device or X.dtype != torch.float32:
            raise ValueError(f"X must be fp32 [K, {self.d_local}] on {self.device}")
        X_in = X
        if isinstance(X, ClientPanels):      # this rank's columns in the panel layout
            ptr, ldx, layout = X.data.data_ptr(), X.panel_stride, _lib.GM_LAYOUT_PANELS
        else:
            if X.stride(1) != 1 or X.data_ptr() % 16 or (X.stride(0) % 4 and X.shape[0] > 1):
                # unit stride and float4-aligned rows, as on every other rank: the AUTO
                # Gram decision is global, so a rank must never fall short of it locally
                X = X.clone(memory_format=torch.contiguous_format)
            ptr, ldx, layout = X.data_ptr(), max(X.stride(0), self.d_local), _lib.GM_LAYOUT_ROWS
        K = X.shape[0]
        guess = opts.get("guess")
        if guess is None:
            raise ValueError("sharded aggregation needs options['guess'] (this rank's shard)")
        g0 = guess.to(device=self.device, dtype=torch.float32).contiguous()
        out = torch.empty(self.d_local, dtype=torch.float32, device=self.device)
        o = _lib.GmOpts()
        o.maxiter = int(opts["maxiter"])
        o.tol = float(opts["tol"])
        o.eps = 1e-4
        o.mode = _lib.GM_MODE_AIRCOMP if aircomp else _lib.GM_MODE_IDEAL
        o.algo = _ALGOS[opts.get("algo", "auto")]
        o.layout = layout
        if not aircomp and opts.get("pre_oma_var") is not None:
            # OMA pre-noise on this rank's columns (keyed by global column: the shards
            # together draw what one unsharded OMA would), fused into the first pass
            if opts.get("pre_oma_seed") is None:
                raise ValueError("sharded pre-noise needs options['pre_oma_seed'] identical on "
                                 "every rank")
            o.pre_oma = 1
            o.pre_oma_var = float(opts["pre_oma_var"])
            o.pre_oma_seed = _seed({"seed": opts["pre_oma_seed"]})
        if aircomp:
            var = opts["noise_var"]
            o.has_noise = int(var is not None)
            o.noise_var = float(var) if var is not None else 0.0
            o.P_max = float(opts["P_max"])
            if _noise_source(opts) != _lib.GM_NOISE_PHILOX:
                raise ValueError("sharded AirComp uses on-device Philox noise")
            if opts.get("seed") is None:
                raise ValueError("sharded AirComp needs options['seed'] identical on every rank")
            o.seed = _seed(opts)
        res = _lib.GmResult()
        with torch.cuda.device(self.device):
            _lib.check(self.ctx.lib.gm_weiszfeld_f32(
                self.ctx.handle, ptr, K, self.d_local, ldx,
                g0.data_ptr(), out.data_ptr(), C.byref(o), C.byref(res),
                torch.cuda.current_stream(self.device).cuda_stream), "gm_weiszfeld_f32")
        self.last_result = _result(res)
        if o.pre_oma and X is not X_in:
            X_in.copy_(X)      # the fused pre-noise is in place on the caller's shard
        return out

    def gm2(self, X, options=None):
        """X: this rank's [K, d_local] columns, as a tensor or a ClientPanels."""
        return self._run(X, options or {}, aircomp=False)

    def gm(self, X, options=None):
        return self._run(X, options or {}, aircomp=True)

    def close(self):
        """Release this rank's context and RCCL communicator (call before
        torch.distributed.destroy_process_group())."""
        self.ctx.close()
