"""Why is the C3 STEP pass slower per byte on a small d-shard?  (round 6, DESIGN.md §4's
shard-width row: 572 us per 1M columns + 27 us on P <= 4, but 11-28 us above that line at
P >= 8.)  The same gm2 call on the first d columns of ONE big panel buffer (a prefix view:
the same allocation as the full C3 matrix) and on a separately allocated copy of exactly
those columns, one JSON line per (d, buffer): the average STEP launch (HIP events).

    python tools/shard_probe.py [--d 11000000 1375232 ...] [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--D", type=int, default=11_000_000, help="columns of the big buffer")
    ap.add_argument("--d", type=int, nargs="+",
                    default=[11_000_000, 2_750_208, 1_375_232, 687_616])
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.panels import ClientPanels
    ctx = bz.context()
    s = torch.cuda.current_stream().cuda_stream
    K, D = a.K, a.D
    big = ClientPanels(K, D)
    X = torch.empty(K, D, device="cuda")
    _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, D, D, K // 5, 0.0, 0.05,
                                           0.25, 0.5, 20211, s), "fill")
    big.copy_rows_(X)
    del X
    g0 = torch.empty(D, device="cuda")
    _lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), D, 0.0, 0.01, 20212, s), "fill")
    torch.cuda.synchronize()

    def view(d, copy):
        p = ClientPanels.__new__(ClientPanels)
        p.K, p.d, p.W = K, d, big.W
        p.npan = -(-d // big.W)
        p.data = big.data[:p.npan].clone() if copy else big.data[:p.npan]
        return p

    for d in a.d:
        for copy in (False, True):
            P = view(d, copy)
            opts = {"maxiter": 1000, "tol": 1e-5, "guess": g0[:d]}
            bz.gm2(P, dict(opts))
            torch.cuda.synchronize()
            ctx.pass_timing(True)
            for _ in range(a.reps):
                bz.gm2(P, dict(opts))
            torch.cuda.synchronize()
            ms, n = ctx.pass_timing(False)
            r = bz.aggregators.last_result
            us = 1e3 * ms / max(n, 1)
            print(json.dumps({"d": d, "buffer": "copy" if copy else "prefix of the 11M buffer",
                              "step_us": us, "us_per_M_columns": us / (d / 1e6),
                              "frac": 4.0 * K * d / (us * 1e-6) / 8e12, "iters": r.iters,
                              "launches": n}), flush=True)
            del P
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
