"""Host logic of the d-sharded (multi-GPU) path, on CPU with gloo, world size 2.

What runs here without a GPU:
  * the shard plan (shard_range): covering, disjoint, 256-aligned;
  * the torch.distributed all-reduce adapter the library calls back into;
  * the decomposition the kernels implement: per-shard partials of
    [D_k^2 | movement^2 | ||g||^2], all-reduced once per Weiszfeld iteration,
    reproduce the unsharded reference gm2 (checked against the oracle).
"""
import ctypes as C
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from byzantine_aircomp_amd.sharded import shard_range, torch_allreduce_adapter
from oracle import aggregators as orc


@pytest.mark.parametrize("d", [1, 255, 256, 7850, 48670, 1_000_001])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_range_partitions(d, world):
    spans = [shard_range(d, world, r) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == d
    for (lo, hi), (lo2, _) in zip(spans, spans[1:]):
        assert hi == lo2 and lo <= hi
    for lo, _ in spans:
        assert lo % 256 == 0 or lo == d


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, fn(rank, world)))
    finally:
        dist.destroy_process_group()


def run_world(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return [out[r] for r in range(world)]


def _adapter_case(rank, world):
    buf = (C.c_double * 5)(*[rank + 1.0 + i for i in range(5)])
    torch_allreduce_adapter()(C.addressof(buf), 5, 0)
    return list(buf)


def test_allreduce_adapter_gloo():
    res = run_world(_adapter_case)
    want = [sum(r + 1.0 + i for r in range(2)) for i in range(5)]
    assert res[0] == want and res[1] == want


def _problem(K=40, d=3000, B=8, seed=11):
    g = torch.Generator().manual_seed(seed)
    p = 0.07 * torch.randn(d, generator=g)
    X = p + 5e-4 * torch.randn(K, d, generator=g)
    X[K - B:] = p + 5e-3 * torch.randn(B, d, generator=g) + 2e-3
    return X, p


def _sharded_weiszfeld(rank, world):
    """The per-iteration exchange of libgmagg's host loop, emulated on CPU."""
    X, p = _problem()
    K, d = X.shape
    lo, hi = shard_range(d, world, rank)
    Xs, g = X[:, lo:hi].double(), p[lo:hi].double()
    part = torch.cat([((Xs - g) ** 2).sum(1), torch.zeros(1), (g ** 2).sum().reshape(1)])
    dist.all_reduce(part)
    iters = 0
    for _ in range(1000):
        iters += 1
        dk = part[:K].sqrt().clamp_min(1e-4)
        w = (1 / dk) / (1 / dk).sum()
        nxt = w @ Xs
        part = torch.cat([((Xs - nxt) ** 2).sum(1), ((g - nxt) ** 2).sum().reshape(1),
                          (nxt ** 2).sum().reshape(1)])
        dist.all_reduce(part)
        g = nxt
        if float(part[K].sqrt()) <= 1e-5:
            break
    return lo, hi, g.float(), iters


def test_sharded_decomposition_matches_reference_gm2():
    res = run_world(_sharded_weiszfeld)
    X, p = _problem()
    want, tr = orc.gm2(X, {"maxiter": 1000, "tol": 1e-5, "guess": p})
    got = torch.zeros_like(want)
    for lo, hi, g, iters in res:
        got[lo:hi] = g
        assert abs(iters - tr.iters) <= 1
    assert float((got - want).norm() / want.norm()) <= 1e-5


def _bad_shard_case(rank, world):
    """A custom shard plan that one rank's library call would refuse (rank 0 ends at a
    column that is not a multiple of 4): ShardedGM validates every rank's shard
    collectively, so EVERY rank raises at construction, before any collective of the
    aggregation (no rank is left waiting in an all-reduce)."""
    from byzantine_aircomp_amd.sharded import ShardedGM
    shard = (0, 1001) if rank == 0 else (1024, 2000)
    try:
        ShardedGM(2000, device=torch.device("cuda", 0), shard=shard)
    except ValueError as e:
        return str(e)
    return None


def test_sharded_bad_shard_raises_on_every_rank():
    res = run_world(_bad_shard_case)
    assert all(r is not None and "hi % 4" in r for r in res)


def test_shard_alignment_rule():
    from byzantine_aircomp_amd.sharded import _aligned
    assert _aligned([(0, 1024), (1024, 2000)], 2000)
    assert _aligned([(256, 512)], 4096)                 # a rehearsal of one rank's shard
    assert not _aligned([(0, 1001)], 2000)              # hi not a multiple of 4
    assert not _aligned([(100, 512)], 2000)             # lo not 256-aligned
    assert _aligned([(0, 1001)], 1001)                  # ragged end of the update
    # world > 1: the shards must tile [0, d_total)
    assert not _aligned([(0, 1024), (768, 2000)], 2000)  # overlap
    assert not _aligned([(0, 768), (1024, 2000)], 2000)  # gap
    assert not _aligned([(0, 1024), (1024, 1536)], 2000)  # short of d_total
    assert _aligned([(1024, 2000), (0, 1024)], 2000)     # any rank order
