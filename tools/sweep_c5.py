"""BASELINE config C5: a draw.ipynb-style Monte-Carlo sweep of independent
aggregations, run as batched launches.

    python tools/sweep_c5.py [--problems 4096] [--K 50] [--d 100000] [--maxiter 1000]

Problems are split evenly over var in {0, 1e-3, 1e-2, 1e-1} (var = 0 -> gm2,
var > 0 -> AirComp gm with Philox noise) and B in {0, 5, 10} Byzantine rows
(~N(0.25, 0.5^2); honest rows ~N(0, 0.05^2)); every problem has its own
seeded data.  Each (var) group is one batched call.  Prints one JSON line per
group and a total (problems/s, aggregations of K x d each).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=4096)
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--d", type=int, default=100_000)
    ap.add_argument("--maxiter", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=1024, help="problems per batched call")
    args = ap.parse_args()
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.batched import gm2_batched, gm_batched

    ctx = bz.context()
    s = torch.cuda.current_stream().cuda_stream
    variances = [0.0, 1e-3, 1e-2, 1e-1]
    per_var = args.problems // len(variances)
    K, d = args.K, args.d
    total_t, total_p = 0.0, 0
    for vi, var in enumerate(variances):
        t_group, n_iter = 0.0, []
        for c0 in range(0, per_var, args.chunk):
            P = min(args.chunk, per_var - c0)
            X = torch.empty(P, K, d, device="cuda")
            for p in range(P):
                B = (0, 5, 10)[(c0 + p) % 3]
                _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X[p].data_ptr(), K, d, d, B,
                                                       0.0, 0.05, 0.25, 0.5,
                                                       1000 * vi + c0 + p, s), "fill")
            g0 = torch.empty(P, d, device="cuda")
            _lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), P * d, 0.0, 0.01,
                                                  777 + vi, s), "fill")
            opts = {"maxiter": args.maxiter, "tol": 1e-5, "guess": g0}
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if var == 0.0:
                _, res = gm2_batched(X, opts)
            else:
                _, res = gm_batched(X, dict(opts, noise_var=var, seed=31 + vi))
            torch.cuda.synchronize()
            t_group += time.perf_counter() - t0
            n_iter += [r.iters for r in res]
            del X, g0
        total_t += t_group
        total_p += per_var
        print(json.dumps({"var": var, "agg": "gm2" if var == 0 else "gm", "problems": per_var,
                          "K": K, "d": d, "seconds": t_group,
                          "problems_per_s": per_var / t_group,
                          "mean_iters": sum(n_iter) / len(n_iter),
                          "GBps_streamed": per_var * (sum(n_iter) / len(n_iter) + 1) * 4.0 * K * d
                          / t_group / 1e9}), flush=True)
    print(json.dumps({"total_problems": total_p, "seconds": total_t,
                      "problems_per_s": total_p / total_t}), flush=True)


if __name__ == "__main__":
    main()
