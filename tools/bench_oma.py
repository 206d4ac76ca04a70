"""OMA (row a4) throughput at the C3 shape on one GPU: in-place per-client AWGN
with on-device Philox draws over K=1000 x d=11M fp32 (8 B of HBM traffic and 2
normals per element).  Prints one JSON line.

    python tools/bench_oma.py [--K 1000] [--d 11000000] [--reps 5]
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
    ap.add_argument("--K", type=int, default=1000)
    ap.add_argument("--d", type=int, default=11_000_000)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import byzantine_aircomp_amd as bz
    X = torch.zeros(a.K, a.d, device="cuda")
    bz.OMA(X, 1e-2, seed=1)                      # warm-up
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    t0 = time.perf_counter()
    for r in range(a.reps):
        bz.OMA(X, 1e-2, seed=2 + r)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    n = a.K * a.d
    print(json.dumps({"op": "OMA philox (gm_oma_philox_f32)", "K": a.K, "d": a.d,
                      "ms_per_call": ms, "wall_ms_per_call": 1e3 * (time.perf_counter() - t0) / a.reps,
                      "elements_per_s": n / (ms * 1e-3),
                      "hbm_GBps_algorithmic": 8.0 * n / (ms * 1e-3) / 1e9,
                      "hbm_frac_of_8TBps": 8.0 * n / (ms * 1e-3) / 8e12}))


if __name__ == "__main__":
    main()
