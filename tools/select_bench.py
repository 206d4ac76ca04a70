"""Time the coordinate-wise order-statistic aggregators (median,
trimmed_mean; M:189-195) on the C3 data recipe, HIP events around each call.

    python tools/select_bench.py [--K 1000 256] [--d 2000000] [--reps 5]

One JSON line per (K, aggregator): ms per call (median of reps) and the HBM rate of the
one read of X it needs.  --layout panels times the same data as ClientPanels.
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
    ap.add_argument("--K", type=int, nargs="+", default=[1000, 256])
    ap.add_argument("--d", type=int, default=2_000_000)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--layout", default="rows", choices=["rows", "panels"],
                    help="the client matrix as the reference's [K, d] stack or as ClientPanels")
    a = ap.parse_args()
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    ctx = bz.context()
    s = torch.cuda.current_stream().cuda_stream
    for K in a.K:
        X = torch.empty(K, a.d, device="cuda")
        _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, a.d, a.d, K // 5, 0.0,
                                               0.05, 0.25, 0.5, 20211, s), "fill")
        Xin = bz.ClientPanels.from_rows(X) if a.layout == "panels" else X
        for name in ("median", "trimmed_mean"):
            fn = getattr(bz, name)
            fn(Xin)
            ts = []
            for _ in range(a.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                fn(Xin)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = statistics.median(ts)
            print(json.dumps({"agg": name, "K": K, "d": a.d, "ms": ms,
                              "GBps": 4.0 * K * a.d / ms / 1e6,
                              "layout": a.layout}), flush=True)
        del X, Xin


if __name__ == "__main__":
    main()
