"""Per-row measurements beside the C3 headline: each row's kernel at a
representative size, device time from HIP events, and the roofline that bounds it.

    python tools/rows_bench.py [--out profiles/rNN_rows.jsonl] [--only a2,f3 ...]

One JSON line per row.  Algorithmic bytes/flops per call are stated in each line
(`bytes` / `flops`); `frac` prices them against HBM 8 TB/s or the dense MFMA /
VALU peak named in `bound`.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

HBM = 8.0e12


def timed(fn, reps=3, warm=1):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps / 1e3          # seconds per call


def fill(ctx, X, B, seed):
    from byzantine_aircomp_amd import _lib
    K, d = X.shape
    _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, B, 0.0, 0.05, 0.25,
                                           0.5, seed, torch.cuda.current_stream().cuda_stream),
               "fill")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    only = set(filter(None, a.only.split(",")))
    import byzantine_aircomp_amd as bz
    ctx = bz.context()
    lines = []

    def emit(d):
        print(json.dumps(d), flush=True)
        lines.append(d)

    def want(r):
        return not only or r in only

    if want("a2"):
        # gm (AirComp) at the C3 shape: it never converges, so the cost
        # is maxiter STEP passes; timed over 20 iterations, priced per pass.
        K, d = 1000, 11_000_000
        X = torch.empty(K, d, device="cuda")
        fill(ctx, X, 200, 20211)
        P = bz.ClientPanels.from_rows(X)
        del X
        g0 = 0.01 * torch.randn(d, device="cuda")
        ctx.pass_timing(True)
        t = timed(lambda: bz.gm(P, {"maxiter": 20, "noise_var": 1e-2, "seed": 7, "guess": g0}),
                  reps=2)
        ms, n = ctx.pass_timing(False)
        per = ms / 1e3 / max(n, 1)
        emit({"row": "a2", "what": "gm AirComp (OMA2 fold + Philox column noise), C3 shape, panels",
              "K": K, "d": d, "iters": bz.aggregators.last_result.iters,
              "s_per_call_20it": t, "pass_us": per * 1e6, "bytes": 4.0 * K * d,
              "bound": "hbm", "frac": 4.0 * K * d / per / HBM,
              "s_per_aggregation_at_1000_it_est": per * 1001})
        del P

    if want("a2r"):
        # gm (AirComp) at the C3 shape on the row-major [K, d] input the reference hands
        # over: >= 64 passes pack a panel copy once (GMAGG_STAGE_PANELS=0: the rows are
        # streamed instead; run both for the A/B); 200 iterations per call
        K, d = 1000, 11_000_000
        X = torch.empty(K, d, device="cuda")
        fill(ctx, X, 200, 20211)
        g0 = 0.01 * torch.randn(d, device="cuda")
        ctx.pass_timing(True)
        t = timed(lambda: bz.gm(X, {"maxiter": 200, "noise_var": 1e-2, "seed": 7, "guess": g0}),
                  reps=2)
        ms, n = ctx.pass_timing(False)
        per = ms / 1e3 / max(n, 1)
        import os
        emit({"row": "a2r", "what": "gm AirComp, C3 shape, rows input, 200 iterations",
              "stage_panels": os.environ.get("GMAGG_STAGE_PANELS", "1") != "0",
              "K": K, "d": d, "iters": bz.aggregators.last_result.iters,
              "s_per_call_200it": t, "pass_us": per * 1e6, "frac": 4.0 * K * d / per / HBM,
              "s_per_aggregation_at_1000_it_est": t * 1001 / 201})
        del X

    if want("a4"):
        K, d = 1000, 11_000_000
        X = torch.zeros(K, d, device="cuda")
        t = timed(lambda: bz.OMA(X, 1e-2, seed=3))
        emit({"row": "a4", "what": "OMA Philox (in place)", "K": K, "d": d, "ms": t * 1e3,
              "bytes": 8.0 * K * d, "bound": "valu (Philox4x32-10 + Box-Muller)",
              "hbm_frac": 8.0 * K * d / t / HBM})
        del X

    if want("f3"):
        K, d = 256, 2_000_000
        X = torch.empty(K, d, device="cuda")
        fill(ctx, X, 51, 99)
        for name, fn, nbytes in (("mean", bz.mean, 4.0 * K * d),
                                 ("median", bz.median, 4.0 * K * d),
                                 ("trimmed_mean", bz.trimmed_mean, 4.0 * K * d)):
            t = timed(lambda: fn(X, {}))
            emit({"row": "f3", "what": name, "K": K, "d": d, "ms": t * 1e3, "bytes": nbytes,
                  "hbm_frac": nbytes / t / HBM})
        Kk, dk = 256, 262_144
        Xk = X[:, :dk].contiguous()
        t = timed(lambda: bz.Krum(Xk, {"honestSize": 205}), reps=3, warm=1)
        pairs = Kk * (Kk + 1) / 2
        emit({"row": "f3", "what": "Krum", "K": Kk, "d": dk, "ms": t * 1e3,
              "flops": 3.0 * pairs * dk, "tflops": 3.0 * pairs * dk / t / 1e12,
              "bytes_min": 4.0 * Kk * dk, "hbm_frac_of_min_bytes": 4.0 * Kk * dk / t / HBM})
        del X, Xk
        # the C3 client count (K = 1000) on a 1M-2M column slice
        K, d = 1000, 2_000_000
        X = torch.empty(K, d, device="cuda")
        fill(ctx, X, 200, 98)
        for name, fn in (("median", bz.median), ("trimmed_mean", bz.trimmed_mean)):
            t = timed(lambda: fn(X, {}))
            emit({"row": "f3", "what": name, "K": K, "d": d, "ms": t * 1e3,
                  "bytes": 4.0 * K * d, "hbm_frac": 4.0 * K * d / t / HBM})
        # the same columns as model weights: tightly clustered around a nonzero value
        # (0.03 +- 0.001 honest), which the selection's candidate compaction reaches later
        X.mul_(0.02).add_(0.03)
        for name, fn in (("median", bz.median), ("trimmed_mean", bz.trimmed_mean)):
            t = timed(lambda: fn(X, {}))
            emit({"row": "f3", "what": name + " (clustered: 0.03 + 0.02 x)", "K": K, "d": d,
                  "ms": t * 1e3, "bytes": 4.0 * K * d, "hbm_frac": 4.0 * K * d / t / HBM})
        X.sub_(0.03).div_(0.02)
        Xk = X[:, :1_000_000].contiguous()
        del X
        t = timed(lambda: bz.Krum(Xk, {"honestSize": 800}), reps=2, warm=1)
        pairs = K * (K + 1) / 2
        emit({"row": "f3", "what": "Krum", "K": K, "d": Xk.shape[1], "ms": t * 1e3,
              "flops": 3.0 * pairs * Xk.shape[1], "tflops": 3.0 * pairs * Xk.shape[1] / t / 1e12})
        del Xk

    if want("c2"):
        K, d = 50, 7850
        X = torch.empty(K, d, device="cuda")
        fill(ctx, X, 10, 5)
        g0 = X.mean(0)
        t = timed(lambda: bz.gm(X, {"maxiter": 1000, "noise_var": 1e-2, "seed": 3, "guess": g0}))
        emit({"row": "a2/C2", "what": "gm AirComp, 1000 iterations, register-resident kernel",
              "K": K, "d": d, "ms_per_aggregation": t * 1e3, "us_per_iteration": t * 1e3,
              "algo": bz.aggregators.last_result.algo})
        t2 = timed(lambda: bz.gm2(X, {"maxiter": 1000, "guess": g0}), reps=10)
        emit({"row": "a1/C1", "what": "gm2 K=50 x 7850", "ms_per_aggregation": t2 * 1e3,
              "iters": bz.aggregators.last_result.iters,
              "algo": bz.aggregators.last_result.algo})

    if a.out:
        with open(a.out, "w") as f:
            for d in lines:
                f.write(json.dumps(d) + "\n")


if __name__ == "__main__":
    main()
