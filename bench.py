"""Benchmark: geometric-median aggregations/sec at K=1000, d=11M (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...     (the driver's N>1 form)

One step = one full `gm2` aggregation (BASELINE config C3): the initial
distance pass plus Weiszfeld iterations until the reference's tol test
(||g_t - g_{t+1}|| <= 1e-5) fires, on a synthetic K=1000 x d=11M fp32 client
matrix already resident in HBM (honest rows ~ N(0, 0.05^2), the last 20% ~
N(0.25, 0.5^2), guess ~ N(0, 0.01^2); generated on the device by Philox).

N > 1: d is sharded over the ranks (256-aligned contiguous column shards),
each Weiszfeld iteration all-reduces a (K+2)-vector of fp64 partials over RCCL
(xGMI), every rank takes the same stop decision; total work is fixed, so
scaling is "strong".  value = aggregations/s of the whole job.

Rank 0 prints ONE JSON line.  `roofline` prices the dominant kernel (the fused
streaming pass: 4*K*d_local algorithmic bytes per launch) with HIP events the
library records around every launch on its stream; `cpu_baseline` times the
CPU oracle (an op-for-op PyTorch-CPU restatement of the reference's gm2) on a
bounded sample on this host.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)

WORKLOADS = {
    # name: (K, d, byzantine rows)
    "c3": (1000, 11_000_000, 200),
    "c3-small": (1000, 1_000_000, 200),
    "c4-shard": (256, 15_625_000, 51),     # one GPU's shard of K=256 x d=125M
    "c5-problem": (50, 100_000, 10),
    "c2": (50, 7850, 10),                   # MNIST MLP d, K=50, B=10 (use --agg gm --var 1e-2)
}
MFMA_F32_PEAK_TFLOPS = 157.3                 # v_mfma_f32_32x32x2_f32, dense (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2516.6               # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz, dense


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=3)
    p.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    p.add_argument("--algo", default="auto", choices=["auto", "stream", "twopass", "gram", "gram_f32"])
    p.add_argument("--agg", default="gm2", choices=["gm2", "gm"])
    p.add_argument("--var", type=float, default=None, help="gm noise variance (None = no AWGN)")
    p.add_argument("--maxiter", type=int, default=1000)
    p.add_argument("--layout", default="auto", choices=["auto", "rows", "panels"],
                   help="client matrix layout: rows = the reference's [K, d] stack; panels = "
                        "ClientPanels [ceil(d/W)][K][W] (streaming algorithm); auto = panels "
                        "for the streaming workloads (c3), rows otherwise.  The other layout "
                        "is timed too (alt_layout in the JSON line).")
    p.add_argument("--alt-steps", type=int, default=None,
                   help="steps for the other layout's measurement (0 = skip)")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-d", type=int, default=2_000_000, help="CPU sample width")
    p.add_argument("--dist", action="store_true",
                   help="take the multi-rank path (process group, RCCL comm, d-shard) even at "
                        "world size 1: a one-GPU rehearsal of the N>1 code")
    p.add_argument("--rehearse-shard", type=int, default=0, metavar="P",
                   help="with --dist at world size 1: run rank 0's d-shard of a P-GPU job "
                        "(its columns, its per-iteration exchange over a 1-rank communicator): "
                        "the per-rank time of the N=P run minus the cross-GPU all-reduce latency. "
                        "Convergence uses the shard's sums only, so iters may differ from N=P.")
    return p.parse_args()


def shard_range(d, n, r, align=256):
    per = -(-d // n)
    per = -(-per // align) * align
    lo = min(d, r * per)
    return lo, min(d, lo + per)


def pmc_traffic(workload, layout):
    """Per-launch HBM bytes of the STEP pass from the newest committed PMC summary
    (rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same bench workload and
    layout; tools/pmc_summary.py applies the gfx950 FETCH_SIZE x2 correction)."""
    import glob
    import re
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}*.json")))
    for path in reversed(files):
        data = json.load(open(path))
        for name, row in data["kernels"].items():
            m = re.search(r"weiszfeld_pass<([^>]*)>", name)
            if not m:
                continue
            targs = m.group(1).split(", ")        # <V,NW,LPR,R,MODE,SCHED,OCC[,PANEL]>
            panel = len(targs) == 8 and targs[7] == "true"
            if targs[4] == "0" and panel == (layout == "panels"):
                return row["hbm_bytes_per_launch"] / 1e9, os.path.relpath(path, ROOT)
    return None, None


def cpu_baseline(X, g0, iters, d_full):
    """Time the oracle gm2 (PyTorch CPU, op-for-op the reference) on a sample."""
    from oracle import aggregators as orc
    threads = torch.get_num_threads()
    Xc, gc = X.cpu(), g0.cpu()
    t0 = time.perf_counter()
    _, tr = orc.gm2(Xc, {"maxiter": iters, "tol": -1.0, "guess": gc})
    dt = time.perf_counter() - t0
    K, d = Xc.shape
    per_agg_full = dt * (d_full / d)
    return {"value": 1.0 / per_agg_full, "unit": "aggregations/s", "cores": threads,
            "kind": "port",
            "sample": (f"oracle gm2 (torch CPU, {threads} threads) on the first {d} columns "
                       f"of the same K={K} matrix, {iters} Weiszfeld iterations (the GPU's "
                       f"converged count; tol disabled), {dt:.2f} s, extrapolated linearly "
                       f"in d to {d_full}")}


def main():
    args = parse()
    # stdout carries exactly one JSON line: everything else written to fd 1 (RCCL's
    # init banner, library chatter) is sent to stderr; the line goes to the saved fd.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist_path = world > 1 or args.dist
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib

    K, d_total, B = WORKLOADS[args.workload]
    if args.rehearse_shard and (world != 1 or not args.dist):
        raise SystemExit("--rehearse-shard needs --dist at world size 1")
    lo, hi = shard_range(d_total, args.rehearse_shard or world, rank)
    d = hi - lo
    ctx = bz.context(dev)
    if dist_path:
        import torch.distributed as dist
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533"), ("RANK", "0"),
                     ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)      # plain `python bench.py --dist` (rehearsal)
        dist.init_process_group("nccl", device_id=dev)
        ctx.set_shard(d_total, lo)
        uid = [None]
        if rank == 0:
            import ctypes as C
            buf = C.create_string_buffer(128)
            _lib.check(ctx.lib.gm_rccl_get_unique_id(buf), "gm_rccl_get_unique_id")
            uid[0] = buf.raw
        dist.broadcast_object_list(uid, src=0)
        ctx.init_rccl(uid[0], world, rank)

    stream = torch.cuda.current_stream(dev).cuda_stream
    X = torch.empty(K, d, dtype=torch.float32, device=dev)
    _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, B, 0.0, 0.05, 0.25,
                                           0.5, 20211, stream), "fill")
    g0 = torch.empty(d, dtype=torch.float32, device=dev)
    _lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, 20212, stream),
               "fill")
    opts = {"maxiter": args.maxiter, "tol": 1e-5, "guess": g0, "algo": args.algo}
    if args.agg == "gm":
        opts.update(noise_var=args.var, seed=2021)
    agg = bz.gm2 if args.agg == "gm2" else bz.gm
    layout = args.layout
    if layout == "auto":
        layout = "panels" if args.workload.startswith("c3") and args.algo in ("auto", "stream") \
            else "rows"
    panels = None

    def inputs(lay):
        nonlocal panels
        if lay == "rows":
            return X
        if panels is None:
            panels = bz.ClientPanels.from_rows(X)     # same values, panel layout (packed once)
        return panels

    def measure(Xin, steps, warmup):
        """warmup untimed aggregations, then `steps` timed between barriers +
        device syncs; returns (max-over-ranks seconds, pass ms, launches, result)."""
        for _ in range(warmup):
            agg(Xin, opts)
        torch.cuda.synchronize(dev)
        if dist_path:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)
        ctx.pass_timing(True)
        t0 = time.perf_counter()
        for _ in range(steps):
            out = agg(Xin, opts)
        torch.cuda.synchronize(dev)
        if dist_path:
            torch.distributed.barrier()
        t1 = time.perf_counter()
        pass_ms, launches = ctx.pass_timing(False)
        res = bz.aggregators.last_result
        elapsed = t1 - t0
        if dist_path:
            t = torch.tensor([elapsed], device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            elapsed = float(t.item())
        del out
        return elapsed, pass_ms, launches, res

    elapsed, pass_ms, launches, res = measure(inputs(layout), args.steps, args.warmup)
    alt = None
    alt_layout = "rows" if layout == "panels" else "panels"
    alt_steps = args.alt_steps if args.alt_steps is not None else max(3, args.steps // 4)
    if alt_steps > 0 and (alt_layout == "rows" or (args.algo in ("auto", "stream")
                                                   and bz.panel_width(K) > 0)):
        a_el, a_ms, a_n, a_res = measure(inputs(alt_layout), alt_steps, 1)
        a_pass = (a_ms / 1e3) / max(a_n, 1)
        alt = {"layout": alt_layout, "value": alt_steps / a_el, "steps": alt_steps,
               "ms_per_step": 1e3 * a_el / alt_steps, "iters": a_res.iters, "algo": a_res.algo,
               "avg_launch_us": a_pass * 1e6,
               "frac": 4.0 * K * d / a_pass / 1e9 / HBM_PEAK_GBS}
    if panels is not None and layout == "rows":
        panels = None

    if rank == 0:
        per_launch_bytes = 4.0 * K * d
        avg_pass_s = (pass_ms / 1e3) / max(launches, 1)
        achieved = per_launch_bytes / avg_pass_s / 1e9
        traffic, traffic_src = pmc_traffic(args.workload, layout) if world == 1 else (None, None)
        if res.algo in ("gram", "gram_f32"):
            # dominant kernel = the Gram partial: upper-triangle 32x32 tiles of the
            # K-padded Gram, 2 FLOP per MAC, d_local columns; the split kernel issues
            # 4 bf16 MFMAs (hh, hm, mh, mm) per tile and 16 columns.  It also reads X
            # once: price both ceilings and report the binding one.
            kt = 1 if K <= 32 else 2 if K <= 64 else 4 if K <= 128 else 8
            split = res.algo == "gram"
            flops = kt * (kt + 1) / 2 * 1024 * 2.0 * d * (4 if split else 1)
            peak = MFMA_BF16_PEAK_TFLOPS if split else MFMA_F32_PEAK_TFLOPS
            tf = flops / avg_pass_s / 1e12
            gbs = per_launch_bytes / avg_pass_s / 1e9
            mf = {"bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                  "frac": tf / peak, "traffic": None}
            hb = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": gbs / HBM_PEAK_GBS, "traffic": None}
            roof, other = (mf, hb) if mf["frac"] >= hb["frac"] else (hb, mf)
            roof.update({"kernel": ("gram_split_partial (v_mfma_f32_32x32x16_bf16, h+m split, "
                                    "upper-triangle tiles)") if split else
                                   "gram_partial (v_mfma_f32_32x32x2_f32, upper-triangle tiles)",
                         "launches_timed": launches, "avg_launch_us": avg_pass_s * 1e6,
                         "algorithmic_flops_per_launch": flops,
                         "algorithmic_bytes_per_launch": per_launch_bytes,
                         "other_ceiling": other})
        else:
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "traffic_unit": "GB per launch", "traffic_source": traffic_src,
                    "kernel": f"weiszfeld_pass (STEP, {layout})", "launches_timed": launches,
                    "avg_launch_us": avg_pass_s * 1e6,
                    "algorithmic_bytes_per_launch": per_launch_bytes}
        line = {
            "metric": "GM aggregations/sec at K=1000,d=11M; % HBM roofline; 1/2/4/8 GPUs",
            "value": args.steps / elapsed,
            "unit": "aggregations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Philox on device: honest N(0,0.05^2), last 20% N(0.25,0.5^2), "
                    "guess N(0,0.01^2))",
            "config": {"workload": f"{args.workload}: {args.agg} K={K} x d={d_total} fp32, B={B} "
                                   f"Byzantine, tol 1e-5, maxiter {args.maxiter}"
                                   + (f", noise_var {args.var}" if args.agg == "gm" else ""),
                       "K": K, "d": d_total, "byzantine": B, "iters": res.iters,
                       "algo": res.algo, "layout": layout,
                       "parallelism": (f"rehearsal: rank 0 of a d-shard x{args.rehearse_shard} "
                                       f"job on 1 GPU (d_local {d})" if args.rehearse_shard else
                                       f"d-shard x{world}" if dist_path else "none"),
                       "passes_per_aggregation": 2 if res.algo.startswith("gram") else res.iters + 1},
            "roofline": roof,
            "cpu_baseline": None,
            "alt_layout": alt,
        }
        if world == 1 and not args.no_cpu and args.agg == "gm2":
            dc = min(args.cpu_d, d)
            line["cpu_baseline"] = cpu_baseline(X[:, :dc].contiguous(), g0[:dc], res.iters, d_total)
        print(json.dumps(line), file=json_out, flush=True)
    torch.cuda.synchronize(dev)
    ctx.close()                       # RCCL communicator + workspace, before the process group
    if dist_path:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
