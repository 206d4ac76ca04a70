"""Cost model of the register-resident batched kernel (resident_batched.hip) on C5's shape.

    python tools/rb_probe.py [--problems 1024] [--K 50] [--d 100000]

Times gm2_batched on ONE batch of C5 problems (ProblemPanels, the bench's device recipe)
with a fixed number of iterations (tol < 0: the tol test never fires) for maxiter in
{1, 2, 4, 8, 16}, with and without the fused pre-noise, and prints one JSON line per
point plus the least-squares fit time = fixed + maxiter * per_iteration, per problem in
flight (ms / (problems / groups)).  Not product code.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=1024)
    ap.add_argument("--K", type=int, default=50)
    ap.add_argument("--d", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--quick", action="store_true",
                    help="resident gm2 only, maxiter 1 and 16 (the per-iteration price; "
                         "GMAGG_RB_DBG variants of a -DGMK_RB_DBG_VARIANTS build)")
    a = ap.parse_args()
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.batched import ProblemPanels, gm2_batched
    dev = torch.device("cuda", 0)
    ctx = bz.context(dev)
    s = torch.cuda.current_stream(dev).cuda_stream
    P, K, d = a.problems, a.K, a.d
    Pn = ProblemPanels(P, K, d, device=dev)
    tmp = torch.empty(K, d, device=dev)
    for p in range(P):
        _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, tmp.data_ptr(), K, d, d, (0, 5, 10)[p % 3],
                                               0.0, 0.05, 0.25, 0.5, 1000 + p, s), "fill")
        _lib.check(ctx.lib.gm_rows_to_panels_f32(ctx.handle, tmp.data_ptr(), K, d, d,
                                                 Pn.data[p].data_ptr(), Pn.W, Pn.panel_stride, s),
                   "pack")
    g0 = torch.empty(P, d, device=dev)
    _lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), g0.numel(), 0.0, 0.01, 7, s),
               "fill")
    torch.cuda.synchronize()
    pts = []
    algos = ("resident",) if a.quick else ("resident", "stream")
    pres = (None,) if a.quick else (None, 1e-2)
    for algo in algos:
        for pre in pres:
            for n in ((1, 16) if a.quick else (1, 2, 4, 8, 16)):
                opts = {"maxiter": n, "tol": -1.0, "guess": g0, "algo": algo}
                if pre is not None:
                    opts.update(pre_oma_var=pre, pre_oma_seed=5)
                gm2_batched(Pn, opts)                      # warm
                torch.cuda.synchronize()
                best = 1e30
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    out, res = gm2_batched(Pn, opts)
                    torch.cuda.synchronize()
                    best = min(best, time.perf_counter() - t0)
                rec = {"dbg": os.environ.get("GMAGG_RB_DBG", "0"), "algo": algo, "pre_oma": pre, "maxiter": n, "ms": 1e3 * best,
                       "iters": res[0].iters, "algo_used": res[0].algo}
                pts.append(rec)
                print(json.dumps(rec), flush=True)
    for algo in algos:
        for pre in pres:
            xs = [(r["maxiter"], r["ms"]) for r in pts if r["algo"] == algo and r["pre_oma"] == pre]
            n = len(xs)
            mx = sum(x for x, _ in xs) / n
            my = sum(y for _, y in xs) / n
            slope = sum((x - mx) * (y - my) for x, y in xs) / sum((x - mx) ** 2 for x, _ in xs)
            icpt = my - slope * mx
            print(json.dumps({"dbg": os.environ.get("GMAGG_RB_DBG", "0"), "fit": algo, "pre_oma": pre, "fixed_ms": icpt,
                              "per_iteration_ms": slope, "problems": P}), flush=True)


if __name__ == "__main__":
    main()
