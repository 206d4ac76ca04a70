"""Time the single-problem AirComp `gm` (1000 iterations, Philox noise) at several (K, d)
shapes on the register-resident kernel — the C2 shape and the ones around it (the EMNIST
MLP's d = 48,670) — so that tile / placement A/Bs (GMAGG_RES_CFG, GMAGG_RES_XCD) can be
checked beyond C2 (GMAGG_RES_HIER: the XCD-hierarchical gather of grids beyond one XCD).
One JSON line per shape:

    python tools/res_shape_bench.py [--shapes 50x7850,50x20000,50x48670] [--reps 5]
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
    ap.add_argument("--shapes", default="50x7850,40x7850,50x20000,50x48670")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import byzantine_aircomp_amd as bz
    dev = torch.device("cuda", 0)
    for sh in a.shapes.split(","):
        K, d = (int(v) for v in sh.split("x"))
        g = torch.Generator(device=dev).manual_seed(K * 131 + d)
        p = 0.01 * torch.randn(d, generator=g, device=dev)
        X = p + 0.05 * torch.randn(K, d, generator=g, device=dev)
        opts = {"maxiter": 1000, "tol": 1e-5, "guess": p, "noise_var": 1e-2, "seed": 7}
        bz.gm(X, dict(opts))                                   # warm-up
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            bz.gm(X, dict(opts))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1e3 / a.reps
        res = bz.aggregators.last_result
        print(json.dumps({"K": K, "d": d, "ms_per_aggregation": ms, "us_per_iteration": 1e3 * ms / max(res.iters, 1),
                          "algo": res.algo, "iters": res.iters, "exchange": res.exchange,
                          "res_hier": os.environ.get("GMAGG_RES_HIER", "default"),
                          "res_cfg": os.environ.get("GMAGG_RES_CFG", "default"),
                          "res_xcd": os.environ.get("GMAGG_RES_XCD", "default")}), flush=True)


if __name__ == "__main__":
    main()
