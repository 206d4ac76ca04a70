"""Krum (SURVEY §8 row f3, M:197-204): the exact pair-distance path against the Gram
path (round 5) over (K, d), HIP events around each call, on the C3 recipe's shape
(honest N(0, 0.05^2), 20 % Byzantine rows N(0.25, 0.5^2), rows permuted).

    python tools/krum_bench.py [--shapes 64x2097152,256x1048576] [--reps 5]

One JSON line per (K, d, path): ms per call (median), the candidates the Gram path
recomputed, and whether both paths chose the same row.
"""
import argparse
import json
import os
import statistics
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="64x131072,64x1048576,128x262144,128x1048576,"
                                        "256x131072,256x1048576,256x4194304")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import byzantine_aircomp_amd as bz
    Krum = bz.aggregators.Krum
    for sh in a.shapes.split(","):
        K, d = (int(v) for v in sh.split("x"))
        honest = int(0.8 * K)
        g = torch.Generator(device="cuda").manual_seed(K + d)
        X = 0.05 * torch.randn(K, d, device="cuda", generator=g)
        X[honest:] = 0.25 + 0.5 * torch.randn(K - honest, d, device="cuda", generator=g)
        X = X[torch.randperm(K, device="cuda", generator=g)].contiguous()
        idx = {}
        for mode, name in (("0", "exact"), ("1", "gram")):
            os.environ["GMAGG_KRUM"] = mode
            bz.Krum(X, {"honestSize": honest})
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                bz.Krum(X, {"honestSize": honest})
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            idx[name] = Krum.last_index
            print(json.dumps({"K": K, "d": d, "path": name, "ms": statistics.median(ts),
                              "info": Krum.last_info, "index": Krum.last_index,
                              "GBps_one_read": 4.0 * K * d / statistics.median(ts) / 1e6}),
                  flush=True)
        print(json.dumps({"K": K, "d": d, "same_index": idx["exact"] == idx["gram"]}), flush=True)
        del X
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
