"""Two-rank run of the d-sharded aggregation (sharded.ShardedGM), both ranks on
ONE GPU over gloo (RCCL refuses two ranks on one device):

    torchrun --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29611 tools/sharded_2rank.py [--d 1000000]

Each rank generates ITS columns of the C3-recipe client matrix (K = 1000,
shard-aware Philox fill keyed by global column), runs gm2 and Philox gm on its
shard with the library's host loop exchanging (K+2)-vectors through the
torch.distributed callback, and rank 0 compares the gathered aggregate with
one unsharded call on the full matrix.  One JSON line per check on stdout.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--d", type=int, default=1_000_000)
    ap.add_argument("--gm-iters", type=int, default=20)
    args = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dev = torch.device("cuda", 0)              # every rank on the one GPU
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo")
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd.sharded import ShardedGM

    K, d = args.K, args.d
    B = K // 5
    sg = ShardedGM(d, device=dev, transport="torch")
    s = torch.cuda.current_stream(dev).cuda_stream
    lib, h = sg.ctx.lib, sg.ctx.handle
    X = torch.empty(K, sg.d_local, device=dev)
    bz._lib.check(lib.gm_fill_clients_f32(h, X.data_ptr(), K, sg.d_local, sg.d_local, B, 0.0, 0.05,
                                          0.25, 0.5, 20211, s), "fill")
    g0 = torch.empty(sg.d_local, device=dev)
    bz._lib.check(lib.gm_fill_normal_f32(h, g0.data_ptr(), sg.d_local, 0.0, 0.01, 20212, s), "fill")

    cases = [("gm2", {"maxiter": 1000, "tol": 1e-5}),
             ("gm", {"maxiter": args.gm_iters, "tol": 1e-5, "noise_var": 1e-2, "seed": 2021})]
    results = []
    for name, opts in cases:
        for layout in ("rows", "panels"):
            Xin = bz.ClientPanels.from_rows(X) if layout == "panels" else X
            dist.barrier()
            t0 = time.perf_counter()
            out = getattr(sg, name)(Xin, dict(opts, guess=g0))
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            res = sg.last_result
            parts = [None] * world
            dist.all_gather_object(parts, (sg.lo, sg.hi, out.cpu(), res.iters, res.algo))
            results.append((name, layout, opts, parts, dt))
            del Xin
    sg.close()

    if rank == 0:
        full = torch.empty(K, d, device=dev)
        ctx = bz.context(dev)
        bz._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, full.data_ptr(), K, d, d, B, 0.0,
                                                  0.05, 0.25, 0.5, 20211, s), "fill")
        gfull = torch.empty(d, device=dev)
        bz._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, gfull.data_ptr(), d, 0.0, 0.01, 20212,
                                                 s), "fill")
        # the shards are the global matrix's columns (Philox keyed by global column)
        lo, hi = sg.lo, sg.hi
        shard_ok = bool(torch.equal(full[:, lo:hi], X))
        for name, layout, opts, parts, dt in results:
            want = getattr(bz, name)(full, dict(opts, guess=gfull, algo="stream"))
            wres = bz.aggregators.last_result
            got = torch.empty(d)
            for plo, phi, o, _, _ in parts:
                got[plo:phi] = o
            w = want.cpu().double()
            rel = float((got.double() - w).norm() / w.norm())
            line = {"check": f"{name} {layout}", "K": K, "d": d, "world": world,
                    "shards": [[p[0], p[1]] for p in parts], "iters": [p[3] for p in parts],
                    "algos": [p[4] for p in parts], "unsharded_iters": wres.iters,
                    "rel_l2_vs_unsharded": rel, "rank0_seconds": dt,
                    "rank0_shard_equals_global_columns": shard_ok,
                    "ok": rel <= 1e-6 and len(set(p[3] for p in parts)) == 1
                    and abs(parts[0][3] - wres.iters) <= 1 and shard_ok}
            print(json.dumps(line), flush=True)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
