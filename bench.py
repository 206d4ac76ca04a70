"""Benchmark: geometric-median aggregations/sec at K=1000, d=11M (BASELINE.json).

    python bench.py [--gpus N --steps K --warmup W] [--workload c3|c4-shard|c2|...]
    torchrun --nproc-per-node N bench.py --gpus N ...     (the driver's N>1 form)

One step = one full aggregation: for the default workload (BASELINE config C3)
one `gm2` call — the initial distance pass plus Weiszfeld iterations until the
reference's tol test (||g_t - g_{t+1}|| <= 1e-5) fires — on a synthetic
K=1000 x d=11M fp32 client matrix already resident in HBM (honest rows ~
N(0, 0.05^2), the last 20% ~ N(0.25, 0.5^2), guess ~ N(0, 0.01^2); generated on
the device by Philox).  `--workload c2` is BASELINE config C2 (AirComp `gm`,
var 1e-2, K=50 x d=7850, 1000 iterations); `c4-shard` a standalone K=256 x d=15.6M
problem (C4's column count per GPU at N = 8; the d-sharded C4 job itself decides the Gram
guard on the GLOBAL ||g|| and streams); `c4` the whole 128 GB C4 job.

N > 1: d is sharded over the ranks (sharded.ShardedGM: 256-aligned contiguous
column shards), each Weiszfeld iteration all-reduces a (K+2)-vector of fp64
partials over RCCL (xGMI), every rank takes the same stop decision; total work
is fixed, so scaling is "strong".  value = aggregations/s of the whole job.

Rank 0 prints ONE JSON line.  `roofline` prices the dominant kernel (the fused
streaming pass: 4*K*d_local algorithmic bytes per launch) with HIP events the
library records around every launch on its stream, and the whole aggregation
(4*K*d_local*(passes) / ms_per_step); `cpu_baseline` times the CPU oracle (an
op-for-op PyTorch-CPU restatement of the reference's gm2 / gm) on a bounded
sample on this host; `check` is a full-size correctness check of the returned
aggregate (the fp64 Weiszfeld fixed-point step at g, all ranks).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "GM aggregations/sec at K=1000,d=11M; % HBM roofline; 1/2/4/8 GPUs"

WORKLOADS = {
    # name: (K, d, byzantine rows, default aggregator, default noise variance)
    "c3": (1000, 11_000_000, 200, "gm2", None),
    "c3-small": (1000, 1_000_000, 200, "gm2", None),
    "c4-shard": (256, 15_625_000, 51, "gm2", None),     # C4's per-GPU column count, standalone
    "c4": (256, 125_000_000, 51, "gm2", None),          # the whole C4 job (d-sharded over N)
    "c5-problem": (50, 100_000, 10, "gm2", None),
    "c2": (50, 7850, 10, "gm", 1e-2),                   # MNIST MLP d, K=50, B=10, AirComp gm
    "c5": (50, 100_000, 10, "gm2", None),               # the batched sweep (run_c5)
}
C5_VARS = (0.0, 1e-3, 1e-2, 1e-1)
C5_BYZ = (0, 5, 10)
MFMA_F32_PEAK_TFLOPS = 157.3                 # v_mfma_f32_32x32x2_f32, dense (MI355X_MICROARCH.md)
MFMA_BF16_PEAK_TFLOPS = 2516.6               # 256 CU x 4 SIMD x 1024 FLOP/clk x 2.4 GHz, dense


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="default 20 (c5: 2 sweeps)")
    p.add_argument("--warmup", type=int, default=None, help="default 3 (c5: 1 sweep)")
    p.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    p.add_argument("--algo", default="auto", choices=["auto", "stream", "twopass", "gram", "gram_f32"])
    p.add_argument("--agg", default=None, choices=["gm2", "gm"],
                   help="aggregator (default: the workload's — gm2, or gm for c2)")
    p.add_argument("--var", type=float, default=None,
                   help="gm noise variance (default: the workload's; None = no AWGN)")
    p.add_argument("--maxiter", type=int, default=1000)
    p.add_argument("--tol", type=float, default=1e-5,
                   help="the reference's tol (1e-5); < 0 runs maxiter iterations (probes only)")
    p.add_argument("--layout", default="auto", choices=["auto", "rows", "panels"],
                   help="client matrix layout: rows = the reference's [K, d] stack; panels = "
                        "ClientPanels [ceil(d/W)][K][W] (streaming algorithm); auto = panels "
                        "for the streaming workloads (c3), rows otherwise.  The other layout "
                        "is timed too (alt_layout in the JSON line).")
    p.add_argument("--alt-steps", type=int, default=None,
                   help="steps for the other layout's measurement (0 = skip)")
    p.add_argument("--separate-oma", action="store_true",
                   help="c5 prenoise reading: OMA as its own pass instead of fused into gm2's "
                        "first pass (A/B)")
    p.add_argument("--soak", type=float, default=8.0,
                   help="seconds of untimed aggregations after the timed region (0 = none): the "
                        "GPU stays busy long enough for an outside utilisation sampler to see it")
    p.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    p.add_argument("--cpu-d", type=int, default=2_000_000, help="CPU sample width (columns)")
    p.add_argument("--cpu-budget", type=float, default=20.0,
                   help="seconds of CPU work the baseline sample aims for")
    p.add_argument("--no-check", action="store_true", help="skip the full-size correctness check")
    p.add_argument("--dist", action="store_true",
                   help="take the multi-rank path (process group, ShardedGM, RCCL comm) even at "
                        "world size 1: a one-GPU rehearsal of the N>1 code")
    p.add_argument("--rehearse-shard", type=int, default=0, metavar="P",
                   help="with --dist at world size 1: run rank 0's d-shard of a P-GPU job "
                        "(its columns, its per-iteration exchange over a 1-rank communicator): "
                        "the per-rank time of the N=P run minus the cross-GPU all-reduce latency. "
                        "Convergence uses the shard's sums only, so iters may differ from N=P.")
    p.add_argument("--problems", type=int, default=4096, help="c5: problems per sweep")
    p.add_argument("--c5-batch", type=int, default=1024,
                   help="c5: problems per batched call (small batches keep a group's passes "
                        "inside the 256 MiB Infinity Cache)")
    p.add_argument("--reading", default="prenoise", choices=["prenoise", "aircomp"],
                   help="c5: var > 0 as the reference's `--agg gm2 --var v` (OMA pre-noise, then "
                        "gm2; M:351-353) or as the AirComp gm aggregator (M:131-160)")
    p.add_argument("--c5-recipe", default=None, choices=["outlier", "caller"],
                   help="c5 data: 'outlier' = honest N(0,0.05^2), B rows N(0.25,0.5^2), guess "
                        "N(0,0.01^2); 'caller' = the reference's own caller (M:349: the guess is "
                        "the current model p ~ N(0,0.07^2), honest rows p + N(0,(5e-4)^2), B rows "
                        "p + 2e-3 + N(0,(5e-3)^2)).  Default: outlier for the prenoise reading, "
                        "caller for the aircomp reading (on the outlier data the reference's own "
                        "gm diverges to NaN; DESIGN.md §3.6)")
    p.add_argument("--one-gpu", action="store_true",
                   help="N>1 rehearsal on a one-GPU box: every rank on cuda:0, gloo process "
                        "group, the torch all-reduce callback instead of RCCL (timing is not "
                        "a scaling measurement)")
    a = p.parse_args()
    if a.steps is None:
        a.steps = 2 if a.workload == "c5" else 20
    if a.warmup is None:
        a.warmup = 1 if a.workload == "c5" else 3
    return a


def host_cpu_share() -> int:
    """CPUs this process may use: its affinity set, capped by a cgroup CPU quota
    (on the GPU box os.cpu_count() shows the whole machine, not this box's share)."""
    n = len(os.sched_getaffinity(0))
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def pmc_traffic(workload, layout, kernel="weiszfeld_pass", mode="0"):
    """Per-launch HBM bytes of the dominant kernel from the newest committed PMC
    summary (rocprofv3 FETCH_SIZE/WRITE_SIZE passes of this same bench workload
    and layout; tools/pmc_summary.py applies the gfx950 FETCH_SIZE x2 correction)."""
    import glob
    import re
    files = [f for f in glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}_*.json"))]
    files += glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_{workload}.json"))
    if "aircomp" not in workload:    # (r3s3_pmc_c5_aircomp_*: the other C5 reading's pass)
        files = [f for f in files if "aircomp" not in os.path.basename(f)]
    for path in sorted(files, key=profile_order, reverse=True):
        data = json.load(open(path))
        for name, row in data.get("kernels", {}).items():
            if "hbm_bytes_per_launch" not in row:      # (a pass without the traffic summary)
                continue
            if kernel == "weiszfeld_pass":
                m = re.search(r"weiszfeld_pass<([^>]*)>", name)
                if not m:
                    continue
                targs = m.group(1).split(", ")        # <V,NW,LPR,R,MODE,SCHED,OCC[,PANEL]>
                panel = len(targs) == 8 and targs[7] == "true"
                if targs[4] == mode and panel == (layout == "panels"):
                    return row["hbm_bytes_per_launch"] / 1e9, os.path.relpath(path, ROOT)
            elif kernel == "gram_h16_partial":
                m = re.search(r"gram_h16_partial<([^>]*)>", name)
                # <KT, DBG, WS>: WS = log2 of the panel width, 0 for row-major X
                if m and (m.group(1).split(", ")[-1] != "0") == (layout == "panels"):
                    return row["hbm_bytes_per_launch"] / 1e9, os.path.relpath(path, ROOT)
            elif kernel in name:
                return row["hbm_bytes_per_launch"] / 1e9, os.path.relpath(path, ROOT)
    return None, None


def latency_floor(kernel):
    """The newest profiles/r*_latency_floor.json entry for a register-resident kernel
    (its exchange-only time per iteration, measured with the compute phases skipped)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_latency_floor.json")),
                   key=profile_order, reverse=True)
    for path in files:
        data = json.load(open(path))
        if kernel in data:
            return data[kernel], os.path.relpath(path, ROOT)
    return None, None


def profile_order(path):
    """(round, session, suffix) of a profiles/ file name: r0N_* = round 1 session N,
    r2_* / r2a_* / r2b_* ... = round 2 sessions 0 / 1 / 2 ..., r3s2z_* = round 3 session 2
    variant z, r4s1_* = round 4 session 1 — the newest measurement wins, whatever the
    lexical order of the names."""
    import re
    name = os.path.basename(path).split("_")[0]
    m = re.fullmatch(r"r0(\d)", name)
    if m:
        return (1, int(m.group(1)), "")
    m = re.fullmatch(r"r(\d+)s(\d+)([a-z]*)", name)
    if m:
        return (int(m.group(1)), int(m.group(2)), m.group(3))
    m = re.fullmatch(r"r(\d+)([a-z]?)", name)
    if m:
        return (int(m.group(1)), (ord(m.group(2)) - ord("a") + 1) if m.group(2) else 0, "")
    return (0, 0, name)


def columns(src, c0, c1):
    """Columns [c0, c1) of a [K, d] client matrix held as a row-major tensor or in the
    panel layout (ClientPanels: c0 a multiple of the panel width), as a [K, c1 - c0] tensor."""
    if isinstance(src, torch.Tensor):
        return src[:, c0:c1]
    W = src.W
    p0, p1 = c0 // W, -(-c1 // W)
    blk = src.data[p0:p1].permute(1, 0, 2).reshape(src.K, (p1 - p0) * W)
    return blk[:, c0 - p0 * W:c1 - p0 * W]


def fixed_point_step(X, g: torch.Tensor, allreduce=None, cols=1 << 20):
    """fp64 Weiszfeld step at g over this rank's columns (all ranks' sums combined by
    `allreduce`): returns (||T(g) - g||, ||g||) with T the gm2 map (M:174-179).  At a
    converged aggregate ||T(g) - g|| is of the order of the reference's last movement
    (<= tol = 1e-5); a wrong aggregate shows up as a large step.  X: a row-major [K, d]
    tensor or a ClientPanels, read in column slices (bounded fp64 temporaries)."""
    K, d = X.shape
    if not isinstance(X, torch.Tensor):
        cols = max(X.W, cols // X.W * X.W)
    gd = g.double()
    d2 = torch.zeros(K, dtype=torch.float64, device=g.device)
    for c0 in range(0, d, cols):
        c1 = min(d, c0 + cols)
        d2 += ((columns(X, c0, c1).double() - gd[c0:c1]) ** 2).sum(1)
    if allreduce:
        allreduce(d2)
    w = 1.0 / d2.sqrt().clamp_min(1e-4)
    nums = torch.zeros(2, dtype=torch.float64, device=g.device)
    ws = w.sum()
    for c0 in range(0, d, cols):
        c1 = min(d, c0 + cols)
        step = (w[:, None] * (columns(X, c0, c1).double() - gd[c0:c1])).sum(0) / ws
        nums[0] += (step ** 2).sum()
        nums[1] += (gd[c0:c1] ** 2).sum()
    if allreduce:
        allreduce(nums)
    return math.sqrt(float(nums[0])), math.sqrt(float(nums[1]))


def cpu_baseline(X, g0, agg, var, iters, d_full, budget, max_cols):
    """Time the CPU oracle (op-for-op torch-CPU restatement of the reference's gm2 /
    gm, M:131-184) on a bounded sample of the same matrix: the first `max_cols`
    columns, a fixed iteration count (tol disabled), scaled to the full
    aggregation (iters Weiszfeld iterations over d_full columns)."""
    from oracle import aggregators as orc
    threads = host_cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        dc = min(max_cols, X.shape[1])
        if not isinstance(X, torch.Tensor):
            dc = max(X.W, dc // X.W * X.W)
        Xc, gc = columns(X, 0, dc).contiguous().cpu(), g0[:dc].contiguous().cpu()
        fn = (lambda n: orc.gm2(Xc, {"maxiter": n, "tol": -1.0, "guess": gc})) if agg == "gm2" \
            else (lambda n: orc.gm(Xc, {"maxiter": n, "tol": -1.0, "guess": gc, "noise_var": var,
                                        "P_max": 1}))
        t0 = time.perf_counter()
        fn(1)
        t1 = time.perf_counter() - t0
        n = max(1, min(iters - 1, int(budget / max(t1, 1e-6))))
        t0 = time.perf_counter()
        fn(n)
        tn = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    per_iter = tn / n
    per_agg_full = per_iter * iters * (d_full / dc)
    K = X.shape[0]
    return {"value": 1.0 / per_agg_full, "unit": "aggregations/s", "cores": threads,
            "kind": "port", "ms_per_iteration_sample": 1e3 * per_iter,
            "host_cpus_visible": os.cpu_count(),
            "sample": (f"oracle {agg} (torch CPU, {threads} threads = this host's CPU share; "
                       f"os.cpu_count() = {os.cpu_count()}) on the first {dc} columns of the same "
                       f"K={K} matrix: {n} Weiszfeld iterations (tol disabled) in {tn:.2f} s; "
                       f"scaled to {iters} iterations (the GPU's count) and d={d_full}"
                       + ("" if dc == d_full else ", linear in d (extrapolated)"))}


def c5_rank_slice(per_var: int, world: int, rank: int):
    """Rank `rank`'s contiguous share [q0, q1) of a var group's `per_var` problems (the
    first per_var % world ranks take one more)."""
    base, extra = divmod(per_var, world)
    q0 = rank * base + min(rank, extra)
    return q0, q0 + base + (1 if rank < extra else 0)


def c5_seed(vi: int, q: int) -> int:
    """Data seed of problem q of var group vi (its index in the whole sweep, any N)."""
    return 1_000_003 * vi + q


def c5_draw_seed(vi: int, c0: int) -> int:
    """Draw seed of a batched call whose first problem is q = c0 of var group vi: the
    library keys problem p of the call seed + p * SEED_STRIDE (batched.py), so problem q
    is keyed 31 + 1000 vi + q * SEED_STRIDE whichever rank and chunk run it."""
    from byzantine_aircomp_amd.batched import SEED_STRIDE
    return (31 + 1000 * vi + c0 * SEED_STRIDE) % 2 ** 64


def run_c5(args, json_out, rank=0, world=1):
    """BASELINE config C5: a draw.ipynb-style Monte-Carlo sweep of `args.problems`
    independent K=50 x d=100k aggregations over var in {0, 1e-3, 1e-2, 1e-1} x
    B in {0, 5, 10}.  One step = the whole sweep: per var group (problems/4 each,
    in batches of <= 1024) one batched call, and for var > 0 in the `prenoise`
    reading (the reference's `--agg gm2 --var v`, M:351-353) the batched OMA
    pre-noise (M:385-394) first — both inside the timed region.  Inputs are
    regenerated on the device (untimed) before every step, since OMA is in place.

    N > 1 (the sweep's problems sharded over GPUs): rank r runs its
    contiguous share of every var group (c5_rank_slice), each problem keyed by its index
    in the WHOLE sweep, so a problem's data, draws and result do not depend on N; no
    collective on the data path, a gloo barrier and max-over-ranks timing around each
    step: strong scaling, value = the sweep's problems / the slowest rank's time."""
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib
    from byzantine_aircomp_amd.batched import gm2_batched, gm_batched, oma_batched
    local = 0 if args.one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
    K, d, _, _, _ = WORKLOADS["c5"]
    ctx = bz.context(dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    per_var = args.problems // len(C5_VARS)
    q0, q1 = c5_rank_slice(per_var, world, rank)      # this rank's share of every var group
    chunk = max(1, min(args.c5_batch, q1 - q0))
    # the guesses of a chunk are one fill keyed by the problems' index in the whole sweep
    # (a context whose shard offset is that index x d), so they do not depend on N
    gctx = bz.aggregators.Context(dev.index)
    # layout: the batched problems in the panel layout (ProblemPanels: every chunk one
    # contiguous block, as for C3) unless --layout rows; the panels are packed from the
    # row-major fill, untimed
    from byzantine_aircomp_amd.batched import ProblemPanels
    use_panels = args.layout in ("auto", "panels")
    # (var, rows X [P, K, d] or None, g0 [P, d], panels or None).  With panels no row-major
    # copy is kept: each problem is generated into one [K, d] scratch matrix and packed
    # (the sweep's resident footprint is the 82 GB of problems, not twice that)
    groups = []
    tmp = torch.empty(K, d, device=dev) if use_panels else None
    for vi, var in enumerate(C5_VARS):
        for c0 in range(q0, q1, chunk):             # c0: the chunk's first problem in the group
            P = min(chunk, q1 - c0)
            groups.append((vi, var, c0, None if use_panels else torch.empty(P, K, d, device=dev),
                           torch.empty(P, d, device=dev),
                           ProblemPanels(P, K, d, device=dev) if use_panels else None))

    def recipe_of(reading):
        return args.c5_recipe or ("caller" if reading == "aircomp" else "outlier")

    def fill_problem(vi, c0, p, dst, g0p, recipe):
        """Problem p's [K, d] rows into dst (its guess g0p already filled)."""
        B = C5_BYZ[(c0 + p) % 3]
        seed = c5_seed(vi, c0 + p)
        if recipe == "outlier":
            _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, dst.data_ptr(), K, d, d, B, 0.0,
                                                   0.05, 0.25, 0.5, seed, stream), "fill")
        else:      # rows around the current model (the guess): the reference's caller
            _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, dst.data_ptr(), K, d, d, B, 0.0,
                                                   5e-4, 2e-3, 5e-3, seed, stream), "fill")
            dst += g0p

    def fill(reading):
        recipe = recipe_of(reading)
        for vi, var, c0, X, g0, Pn in groups:
            gctx.set_shard(per_var * d, c0 * d)
            _lib.check(ctx.lib.gm_fill_normal_f32(gctx.handle, g0.data_ptr(), g0.numel(), 0.0,
                                                  0.01 if recipe == "outlier" else 0.07,
                                                  777 + vi, stream), "fill")
            for p in range(g0.shape[0]):
                if Pn is None:
                    fill_problem(vi, c0, p, X[p], g0[p], recipe)
                else:
                    fill_problem(vi, c0, p, tmp, g0[p], recipe)
                    _lib.check(ctx.lib.gm_rows_to_panels_f32(
                        ctx.handle, tmp.data_ptr(), K, d, d, Pn.data[p].data_ptr(), Pn.W,
                        Pn.panel_stride, stream), "pack")
        torch.cuda.synchronize(dev)

    outs = {}                        # the last step's aggregates per group (for `check`)

    def step(reading):
        iters, per_group = [], {}
        for vi, var, c0, Xr, g0, Pn in groups:
            X = Pn if Pn is not None else Xr
            opts = {"maxiter": args.maxiter, "tol": args.tol, "guess": g0}
            t0 = time.perf_counter()
            if var == 0.0:
                out, res = gm2_batched(X, opts)
            elif reading == "prenoise" and args.separate_oma:
                oma_batched(X, var, seed=c5_draw_seed(vi, c0))
                out, res = gm2_batched(X, opts)
            elif reading == "prenoise":
                # the pre-noise fused into gm2's first pass (same draws as oma_batched)
                out, res = gm2_batched(X, dict(opts, pre_oma_var=var,
                                               pre_oma_seed=c5_draw_seed(vi, c0)))
            else:
                out, res = gm_batched(X, dict(opts, noise_var=var, seed=c5_draw_seed(vi, c0)))
            outs[(vi, c0)] = (out, res)
            torch.cuda.synchronize(dev)
            dt = time.perf_counter() - t0
            its = [r.iters for r in res]
            iters += its
            g = per_group.setdefault(var, {"seconds": 0.0, "problems": 0, "iters": 0})
            g["seconds"] += dt
            g["problems"] += len(its)
            g["iters"] += sum(its)
        return iters, per_group

    def measure(reading, steps, warmup):
        for _ in range(warmup):
            fill(reading)
            step(reading)
        total, pass_ms, launches, iters, groups_out = 0.0, 0.0, 0, [], {}
        for _ in range(steps):
            fill(reading)
            ctx.pass_timing(True)
            torch.cuda.synchronize(dev)
            if dist is not None:
                dist.barrier()
            t0 = time.perf_counter()
            iters, groups_out = step(reading)
            torch.cuda.synchronize(dev)
            el = time.perf_counter() - t0
            if dist is not None:
                t = torch.tensor([el], dtype=torch.float64)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                el = float(t[0])
            total += el
            ms, n = ctx.pass_timing(False)
            pass_ms += ms
            launches += n
        return total, pass_ms, launches, iters, groups_out

    total, pass_ms, launches, iters, per_group = measure(args.reading, args.steps, args.warmup)
    check = c5_check(groups, outs, args.reading, args.maxiter, recipe_of(args.reading)) \
        if not args.no_check else None
    n_prob = len(iters)                          # this rank's problems
    n_total = per_var * len(C5_VARS)             # the sweep's, over every rank
    mean_it = sum(iters) / n_prob
    step_bytes = sum(iters) * 4.0 * K * d            # algorithmic STEP-pass bytes per sweep
    achieved = step_bytes * args.steps / (pass_ms / 1e3) / 1e9 if pass_ms > 0 else None
    agg_bytes = sum(i + 1 for i in iters) * 4.0 * K * d
    alt_reading = "aircomp" if args.reading == "prenoise" else "prenoise"
    alt = None
    if args.alt_steps != 0 and world == 1:
        a_total, _, _, a_iters, a_groups = measure(alt_reading, 1, 0)
        alt = {"reading": alt_reading, "recipe": recipe_of(alt_reading),
               "value": len(a_iters) / a_total, "seconds": a_total,
               "mean_iters": sum(a_iters) / len(a_iters),
               "groups": {str(k): {"problems_per_s": v["problems"] / v["seconds"],
                                   "mean_iters": v["iters"] / v["problems"]}
                          for k, v in a_groups.items()}}
    algo_used = outs[(groups[0][0], groups[0][2])][1][0].algo
    if algo_used == "resident":
        # the register-resident batched kernel reads each problem's X once (and, in the
        # prenoise reading, writes the noised copy back once): price THOSE bytes; the
        # iterations run on chip, so the kernel is bound by the exchange latency per
        # iteration, and `streaming_equivalent` is the streaming algorithm's bytes over
        # the same time (it exceeds the HBM peak when the residency pays)
        hbm_bytes = sum(((2 if (args.reading == "prenoise" and var > 0) else 1)
                         * g0.shape[0] * 4.0 * K * d) for _, var, _, _, g0, _ in groups)
        per_launch = hbm_bytes / max(launches / max(args.steps, 1), 1)
        # (each reading quotes the PMC pass of its own launches: the prenoise reading's
        # gm2 kernel, the aircomp reading's gm kernel — the launch that dominates the sweep)
        traffic, traffic_src = (pmc_traffic("c5", "panels" if use_panels else "rows",
                                            kernel="weiszfeld_resident_batched<50, 32, 0")
                                if args.reading == "prenoise" else
                                pmc_traffic("c5-aircomp", "panels" if use_panels else "rows",
                                            kernel="weiszfeld_resident_batched<50, 32, 1"))
        achieved = hbm_bytes * args.steps / (pass_ms / 1e3) / 1e9 if pass_ms > 0 else None
        # The kernel is latency-bound: each iteration is a cross-CU exchange of every block's
        # partials plus the phases' VALU work, with the problem's tile on chip.  Roofline =
        # time per iteration of one problem in flight (a group of NB blocks) against the
        # exchange floor (the same kernel with its compute phases skipped; profiles/),
        # the tile load's fixed cost per problem (profiled) taken out first.
        fl, fl_src = latency_floor("weiszfeld_resident_batched")
        ng = fl["groups"] if fl else None
        it_us = None
        if fl and pass_ms > 0:
            probs = len(iters)
            t_step_us = 1e3 * pass_ms / args.steps
            it_us = (t_step_us * ng / probs - fl["fixed_us_per_problem"]) / (sum(iters) / probs)
        roofline = {
            "bound": "latency", "unit": "us per iteration (one problem in flight)",
            "achieved": it_us, "peak": fl["exchange_floor_us_per_iteration"] if fl else None,
            "frac": fl["exchange_floor_us_per_iteration"] / it_us if fl and it_us else None,
            "frac_def": "exchange floor / achieved time per iteration (<= 1; time-like: the floor "
                        "is the fastest an iteration can be with this exchange)",
            "floor_source": fl_src,
            "achieved_def": "(summed kernel time per sweep x groups / problems - the profiled fixed "
                            "cost per problem: tile load, INIT, last gather) / mean iterations",
            "kernel": "weiszfeld_resident_batched (each problem's X read once, held in VGPRs + "
                      "LDS for all its iterations)",
            "launches_timed": launches, "avg_launch_us": 1e3 * pass_ms / max(launches, 1),
            "traffic": traffic, "traffic_unit": "GB per launch (one 1024-problem group, PMC)",
            "traffic_algorithmic": per_launch / 1e9, "traffic_source": traffic_src,
            "hbm_tile_load": {
                "bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                "achieved": fl.get("tile_load_hbm_GBs") if fl else None,
                "frac": fl["tile_load_hbm_GBs"] / HBM_PEAK_GBS if fl else None,
                "source": fl.get("tile_load_note") if fl else None,
                "kernel_bytes_over_kernel_time_GBs": achieved,
                "kernel_bytes_def": "4*K*d per problem (one read of X) + 4*K*d per problem of the "
                                    "prenoise groups (the noised X written back), / summed kernel "
                                    "time (iterations included: not an HBM rate of the loads)"},
            "streaming_equivalent_frac": agg_bytes / (total / args.steps) / 1e9 / HBM_PEAK_GBS,
            "streaming_equivalent_def": "sum_p 4*K*d*(iters_p+1) / ms_per_step / 8 TB/s: the bytes "
                                        "the streaming path would move, over the sweep's time (a "
                                        "comparison with streaming, not a roofline)"}
    else:
        traffic, traffic_src = pmc_traffic("c5", "panels" if use_panels else "rows")
        roofline = {
            "bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS if achieved else None, "traffic": traffic,
            "traffic_unit": "GB per batched STEP launch with every problem of a "
                            f"{chunk}-problem group active (PMC of the AirComp reading)",
            "traffic_algorithmic": chunk * 4.0 * K * d / 1e9 if traffic else None,
            "traffic_source": traffic_src,
            "kernel": "weiszfeld_pass (batched STEP, blockIdx.y = problem)",
            "launches_timed": launches, "avg_launch_us": 1e3 * pass_ms / max(launches, 1),
            "algorithmic_bytes": "4*K*d per problem per Weiszfeld iteration (sum over "
                                 "problems of iters) / summed STEP launch time",
            "aggregation_frac": agg_bytes / (total / args.steps) / 1e9 / HBM_PEAK_GBS,
            "aggregation_frac_def": "sum_p 4*K*d*(iters_p+1) / ms_per_step / 8 TB/s "
                                    "(OMA pre-noise time included, its bytes not)"}
    cpu = None
    if not args.no_cpu and world == 1:
        vi0, _, c00, X0, g00, _ = groups[0]
        if X0 is None:                       # problem 0's clean rows, regenerated
            fill_problem(vi0, c00, 0, tmp, g00[0], recipe_of(args.reading))
            torch.cuda.synchronize(dev)
        cpu = c5_cpu_baseline(tmp if X0 is None else X0[0], g00[0], mean_it, n_prob,
                              args.cpu_budget)
    line = {
        "metric": METRIC, "value": n_total * args.steps / total, "unit": "aggregations/s",
        "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * total / args.steps, "higher_is_better": True,
        "scaling": "strong" if world > 1 else "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": ("synthetic (Philox on device: honest N(0,0.05^2), B rows N(0.25,0.5^2), "
                 "guess N(0,0.01^2))" if recipe_of(args.reading) == "outlier" else
                 "synthetic (Philox on device, the reference's caller M:349: guess = model p ~ "
                 "N(0,0.07^2), honest rows p + N(0,(5e-4)^2), B rows p + 2e-3 + N(0,(5e-3)^2))"),
        "config": {"workload": f"c5: {n_total} independent gm2 problems K={K} x d={d} fp32 over "
                               f"var {list(C5_VARS)} x B {list(C5_BYZ)}, reading '{args.reading}'"
                               + ((" (OMA pre-noise then gm2, M:351-353; separate OMA pass)"
                                   if args.separate_oma else
                                   " (OMA pre-noise then gm2, M:351-353; the pre-noise fused "
                                   "into gm2's first pass)")
                                  if args.reading == "prenoise" else " (AirComp gm for var > 0)"),
                   "K": K, "d": d, "problems": n_total, "problems_per_rank": n_prob,
                   "mean_iters": mean_it, "batch": chunk,
                   "algo": algo_used, "recipe": recipe_of(args.reading),
                   "parallelism": ("register-resident batched (one launch per group: each problem "
                                   "held on chip for all its iterations)" if algo_used == "resident"
                                   else "batched (one launch per pass covers every problem of a group)")
                                  + (f"; the sweep's problems sharded over {world} GPUs (rank 0: "
                                     f"{n_prob}; no data-path collective)" if world > 1 else ""),
                   "layout": "panels (ProblemPanels)" if use_panels else "rows",
                   "groups": {str(k): {"problems_per_s": v["problems"] / v["seconds"],
                                       "mean_iters": v["iters"] / v["problems"]}
                              for k, v in per_group.items()}},
        "roofline": roofline,
        "cpu_baseline": cpu,
        "check": dict(check or {}, max_iters=max(iters), min_iters=min(iters)),
        "alt_layout": alt,
    }
    print(json.dumps(line), file=json_out, flush=True)


def c5_check(groups, outs, reading, maxiter, recipe, per_group=3):
    """Full-size correctness of the last timed sweep.

    gm2 groups (var = 0, and every group of the prenoise reading): for the first, middle
    and last problem, the fp64 gm2 fixed-point step ||T(g) - g|| (T = M:174-179) at the
    returned aggregate over that problem's (noisy, for the prenoise reading) K x d matrix
    as the kernels read it; the reference stops at movement <= tol = 1e-5, a wrong
    aggregate shows up as a large step.

    AirComp gm groups (never converge, 1000 iterations): the fraction of problems with a
    finite aggregate, and the distance of each aggregate from the ideal GM of the same
    problem (gm2_batched, untimed) — the AirComp error a draw.ipynb-style sweep plots.
    The reference's own gm is unstable once sqrt(var d / 2) exceeds K / (sqrt(500) s)
    (s = RMS of the iterate; its noise then outgrows the distances that scale the signal,
    DESIGN.md §3.6): at d = 100k, s = 0.07 that is var ~ 0.02, so the var = 0.1 group
    diverges in the reference too (tests/test_oracle_c5_stability.py); `ok` requires
    finite aggregates in the groups below the bound only.  The kernel is pinned to
    oracle.gm over 1000 iterations by tests/test_gpu_c5_fullsize.py."""
    from byzantine_aircomp_amd.batched import gm2_batched
    worst, worst_rel, n, ok_air = 0.0, 0.0, 0, True
    air = {}
    for vi, var, c0, Xr, g0, Pn in groups:
        out, res = outs[(vi, c0)]
        P = out.shape[0]
        if reading == "aircomp" and var > 0:
            X = Pn if Pn is not None else Xr
            ideal, _ = gm2_batched(X, {"maxiter": maxiter, "tol": 1e-5, "guess": g0})
            fin = torch.isfinite(out).all(dim=1)
            rel_all = (out - ideal).norm(dim=1) / ideal.norm(dim=1)
            # a trajectory that ran away can stay finite for a while: "stable" = finite and
            # within half the GM's norm of it
            stable = fin & (rel_all < 0.5)
            a = air.setdefault(str(var), {"problems": 0, "finite": 0, "stable": 0,
                                          "rel_to_gm2": []})
            a["problems"] += P
            a["finite"] += int(fin.sum())
            a["stable"] += int(stable.sum())
            a["rel_to_gm2"] += rel_all[stable].tolist()
            if recipe == "outlier" or _c5_stable(var, X):
                ok_air &= bool(stable.all())
            continue
        for p in sorted({0, P // 2, P - 1})[:per_group]:
            if Pn is not None:
                Xp = Pn.data[p].permute(1, 0, 2).reshape(Pn.K, Pn.npan * Pn.W)[:, :Pn.d]
            else:
                Xp = Xr[p]
            step, gn = fixed_point_step(Xp, out[p])
            worst = max(worst, step)
            worst_rel = max(worst_rel, step / max(gn, 1e-300))
            n += 1
    out = {"what": "gm2 groups: fp64 gm2 step ||T(g) - g|| / ||g|| at the returned g of the "
                   "first, middle and last problem of every group, over the problem's full K x d "
                   "matrix (noisy for the prenoise reading); T = M:174-179",
           "problems_checked": n, "max_fixed_point_step": worst, "max_relative_step": worst_rel,
           "ok": ok_air and worst <= 1e-4}
    if air:
        out["aircomp_groups"] = {
            k: {"finite_frac": v["finite"] / v["problems"],
                "stable_frac": v["stable"] / v["problems"],
                "mean_rel_to_gm2": (sum(v["rel_to_gm2"]) / len(v["rel_to_gm2"])
                                    if v["rel_to_gm2"] else None),
                "max_rel_to_gm2": max(v["rel_to_gm2"]) if v["rel_to_gm2"] else None,
                "noise_ratio_r": _c5_ratio(float(k), groups[0][5] or groups[0][3]),
                "stable_regime": recipe == "caller" and _c5_stable(float(k), groups[0][5]
                                                                   or groups[0][3])}
            for k, v in air.items()}
        out["aircomp_what"] = ("AirComp gm groups: over every problem the fraction finite and the "
                               "fraction stable (finite and within 0.5 ||g_gm2|| of the ideal GM of "
                               "the same problem), and ||g_gm - g_gm2|| / ||g_gm2|| over the stable "
                               "ones.  The reference's gm adds column noise of norm ~ r d_k per "
                               "iteration, r = sqrt(var d / 2) sqrt(500) s / K (s = 0.07, the model's "
                               "RMS): stable at r = 0.22 (var 1e-3), marginal at 0.70 (1e-2: whether "
                               "a trajectory runs away is decided by rounding), divergent at 2.2 "
                               "(1e-1); `ok` requires every problem stable where r < 0.5 "
                               "(DESIGN.md §3.6, tests/test_oracle_c5_stability.py)")
    return out


def _c5_ratio(var, X, s=0.07):
    """The reference gm's noise ratio on the caller recipe: r = sqrt(var d / 2) sqrt(500) s / K
    (s = the model's RMS, 0.07)."""
    K, d = (X.shape[1], X.shape[2]) if isinstance(X, torch.Tensor) else (X.K, X.d)
    return math.sqrt(var * d / 2) * math.sqrt(500.0) * s / K


def _c5_stable(var, X):
    """Measured stable regime of the reference's gm on the caller recipe: r < 0.5 (r = 0.22
    stable, 0.70 marginal)."""
    return _c5_ratio(var, X) < 0.5


def c5_cpu_baseline(X, g0, mean_iters, problems, budget):
    """Oracle gm2 (op-for-op torch-CPU restatement of M:162-184) on ONE C5 problem
    (K=50 x d=100k, the same data as GPU problem 0), tol disabled, a bounded number
    of iterations; scaled to the sweep's mean iteration count x its problem count
    (the OMA pre-noise of the var > 0 groups is not added: the CPU figure is a
    lower bound on the reference's time)."""
    from oracle import aggregators as orc
    threads = host_cpu_share()
    prev = torch.get_num_threads()
    torch.set_num_threads(threads)
    try:
        Xc, gc = X.cpu(), g0.cpu()
        t0 = time.perf_counter()
        orc.gm2(Xc, {"maxiter": 1, "tol": -1.0, "guess": gc})
        t1 = time.perf_counter() - t0
        n = max(1, min(200, int(budget / max(t1, 1e-6))))
        t0 = time.perf_counter()
        orc.gm2(Xc, {"maxiter": n, "tol": -1.0, "guess": gc})
        tn = time.perf_counter() - t0
    finally:
        torch.set_num_threads(prev)
    per_problem = tn / n * (mean_iters + 1)
    return {"value": 1.0 / per_problem, "unit": "aggregations/s", "cores": threads, "kind": "port",
            "host_cpus_visible": os.cpu_count(),
            "sample": f"oracle gm2 (torch CPU, {threads} threads) on one K=50 x d=100000 problem: "
                      f"{n} iterations in {tn:.2f} s; scaled to {mean_iters + 1:.2f} passes per "
                      f"problem (the sweep's mean); {problems} problems take {problems * per_problem:.0f} s"}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n: int, argv, cmd=None, poll_s: float = 0.2) -> int:
    """`python bench.py --gpus N` with N > 1 and no launcher around it (no WORLD_SIZE in
    the environment): start N fresh worker processes of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR (127.0.0.1) /
    MASTER_PORT set — exactly what `torch.distributed.run --nproc-per-node N` gives them —
    relay rank 0's one JSON line to stdout, and return non-zero if any rank fails (the
    other ranks are then stopped, by their own PIDs, so none waits at a barrier forever).
    This process makes no GPU call: it only spawns and waits.  `cmd` replaces the worker
    command line (tests)."""
    import subprocess
    import tempfile
    cmd = cmd or [sys.executable, os.path.abspath(__file__), *argv]
    port = free_port()
    procs = []
    # rank 0's stdout goes to a file, read once every rank has exited (a pipe read only at
    # the end would block a rank that writes more than the pipe holds)
    out0 = tempfile.TemporaryFile()
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=out0 if r == 0 else
                                      subprocess.DEVNULL))
    rc = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            c = procs[r].poll()
            if c is None:
                continue
            live.discard(r)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"bench.py launcher: rank {r} exited with {c}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in live:
                    procs[q].terminate()
        if live:
            time.sleep(poll_s)
    for p in procs:
        p.wait()
    out0.seek(0)
    out = out0.read().decode(errors="replace")
    out0.close()
    lines = [ln for ln in out.splitlines() if ln.strip()]
    if lines:
        sys.stdout.write(lines[-1] + "\n")
        sys.stdout.flush()
    elif rc == 0:
        print("bench.py launcher: rank 0 printed no result line", file=sys.stderr)
        rc = 1
    return rc


def visible_gpus():
    """GPUs this process could open, counted WITHOUT any GPU-library call (the launcher
    parent must not initialise a GPU runtime before it spawns the ranks): the KFD topology's
    GPU nodes (gpu_id != 0), narrowed by HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES /
    CUDA_VISIBLE_DEVICES when set.  None when the topology cannot be read."""
    import glob
    n = 0
    try:
        for node in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id"):
            with open(node) as f:
                n += int(f.read().strip() or "0") != 0
    except (OSError, ValueError):
        return None
    if n == 0:
        return None
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip()]))
    return n


def main():
    args = parse()
    if args.workload == "c5" and args.problems // len(C5_VARS) < args.gpus:
        # every rank takes a contiguous share of each var group: no empty ranks
        raise SystemExit(f"c5: --problems {args.problems} gives {args.problems // len(C5_VARS)} "
                         f"problems per var group, fewer than --gpus {args.gpus}")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # the driver's plain `python bench.py --gpus N`: become the launcher.  No GPU-library
        # call here (not even a device count): the GPUs are counted from the KFD topology, and
        # where that is unreadable the ranks find out themselves and fail loudly
        n_vis = None if args.one_gpu else visible_gpus()
        if n_vis is not None and n_vis < args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but {n_vis} GPU(s) visible")
        raise SystemExit(launch_ranks(args.gpus, sys.argv[1:]))
    if os.environ.get("BENCH_EXIT_MAPS"):
        # diagnostics: this process's memory map as the interpreter exits, to attribute
        # the PCs of a crash in the C-level exit handlers to their DSOs
        import atexit
        path = os.environ["BENCH_EXIT_MAPS"]
        atexit.register(lambda: open(path, "w").write(open("/proc/self/maps").read()))
    # stdout carries exactly one JSON line: everything else written to fd 1 (RCCL's
    # init banner, library chatter) is sent to stderr; the line goes to the saved fd.
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.workload == "c5":
        if world != args.gpus:
            raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
        run_c5(args, json_out if rank == 0 else open(os.devnull, "w"), rank, world)
        if world > 1:
            import torch.distributed as dist
            dist.destroy_process_group()
        return
    local = 0 if args.one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist_path = world > 1 or args.dist or args.one_gpu
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    import byzantine_aircomp_amd as bz
    from byzantine_aircomp_amd import _lib

    K, d_total, B, agg_name, var = WORKLOADS[args.workload]
    agg_name = args.agg or agg_name
    if args.var is not None:
        var = args.var
    if args.rehearse_shard and (world != 1 or not args.dist):
        raise SystemExit("--rehearse-shard needs --dist at world size 1")
    stream = torch.cuda.current_stream(dev).cuda_stream
    sg = None
    allreduce = None
    if dist_path:
        import torch.distributed as dist
        from byzantine_aircomp_amd.sharded import ShardedGM, shard_range
        for k, v in (("MASTER_ADDR", "127.0.0.1"), ("MASTER_PORT", "29533"), ("RANK", "0"),
                     ("WORLD_SIZE", "1")):
            os.environ.setdefault(k, v)      # plain `python bench.py --dist` (rehearsal)
        if args.one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        shard = shard_range(d_total, args.rehearse_shard, 0) if args.rehearse_shard else None
        # the aggregation's own context (RCCL comm + this rank's shard), never the
        # process-wide per-device one
        sg = ShardedGM(d_total, device=dev, transport="torch" if args.one_gpu else "rccl",
                       shard=shard)
        ctx = sg.ctx
        lo, hi = sg.lo, sg.hi

        def allreduce(t):
            dist.all_reduce(t)
    else:
        ctx = bz.context(dev)
        lo, hi = 0, d_total
    d = hi - lo

    layout = args.layout
    if layout == "auto":
        layout = "panels" if (args.workload.startswith("c3") and args.algo in ("auto", "stream")) \
            or (args.workload.startswith("c4") and args.algo in ("auto", "stream", "gram")) \
            else "rows"
    # a panel-layout input whose row-major copy would not fit beside it (the whole C4 job,
    # 256 x 125M = 128 GB, on one GPU) is generated straight into the panels, column slice
    # by column slice through a scratch matrix: no rows copy, no rows-layout measurement
    big = layout == "panels" and 8.0 * K * d > 120e9
    panels = None
    if big:
        panels = bz.ClientPanels(K, d, device=dev)
        S = panels.W * 8192
        tmp = torch.empty(K, S, dtype=torch.float32, device=dev)
        fctx = bz.aggregators.Context(dev.index)       # its shard offset keys the columns
        for c0 in range(0, d, S):
            n = min(S, d - c0)
            fctx.set_shard(d_total, lo + c0)
            _lib.check(ctx.lib.gm_fill_clients_f32(fctx.handle, tmp.data_ptr(), K, n, S, B, 0.0,
                                                   0.05, 0.25, 0.5, 20211, stream), "fill")
            _lib.check(ctx.lib.gm_rows_to_panels_f32(fctx.handle, tmp.data_ptr(), K, n, S,
                                                     panels.data[c0 // panels.W].data_ptr(),
                                                     panels.W, panels.panel_stride, stream), "pack")
        torch.cuda.synchronize(dev)
        fctx.close()
        del tmp
        X = None
    else:
        X = torch.empty(K, d, dtype=torch.float32, device=dev)
        _lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, B, 0.0, 0.05,
                                               0.25, 0.5, 20211, stream), "fill")
    g0 = torch.empty(d, dtype=torch.float32, device=dev)
    _lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, 20212, stream),
               "fill")
    opts = {"maxiter": args.maxiter, "tol": args.tol, "guess": g0, "algo": args.algo}
    if agg_name == "gm":
        opts.update(noise_var=var, seed=2021)
    if sg is not None:
        agg = sg.gm2 if agg_name == "gm2" else sg.gm

        def last():
            return sg.last_result
    else:
        agg = bz.gm2 if agg_name == "gm2" else bz.gm

        def last():
            return bz.aggregators.last_result
    def inputs(lay):
        nonlocal panels
        if lay == "rows":
            return X
        if panels is None:
            panels = bz.ClientPanels.from_rows(X)     # same values, panel layout (packed once)
        return panels

    def measure(Xin, steps, warmup):
        """warmup untimed aggregations, then `steps` timed between barriers +
        device syncs; returns (max-over-ranks seconds, pass ms, launches, result, out)."""
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
        res = last()
        elapsed = t1 - t0
        if dist_path:
            t = torch.tensor([elapsed], dtype=torch.float64,
                             device="cpu" if args.one_gpu else dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            elapsed = float(t.item())
        return elapsed, pass_ms, launches, res, out

    elapsed, pass_ms, launches, res, out = measure(inputs(layout), args.steps, args.warmup)
    passes = 2 if res.algo.startswith("gram") else res.iters + 1
    # untimed soak: the same aggregation repeated for ~args.soak seconds (a count every
    # rank derives from the max-over-ranks time, so collectives stay in lockstep)
    soak = None
    if args.soak > 0:
        n_soak = int(args.soak / max(elapsed / args.steps, 1e-6))
        t0 = time.perf_counter()
        for _ in range(n_soak):
            agg(inputs(layout), opts)
        torch.cuda.synchronize(dev)
        soak = {"aggregations": n_soak, "seconds": time.perf_counter() - t0,
                "note": "untimed, after the timed region (GPU-busy signal for outside samplers)"}
    alt = None
    alt_layout = "rows" if layout == "panels" else "panels"
    alt_steps = args.alt_steps if args.alt_steps is not None else max(3, args.steps // 4)
    if alt_steps > 0 and not big and (alt_layout == "rows" or (args.algo in ("auto", "stream", "gram")
                                                   and bz.panel_width(K) > 0
                                                   and d_total >= 1 << 20)):
        a_el, a_ms, a_n, a_res, _ = measure(inputs(alt_layout), alt_steps, 1)
        a_pass = (a_ms / 1e3) / max(a_n, 1)
        a_passes = 2 if a_res.algo.startswith("gram") else a_res.iters + 1
        alt = {"layout": alt_layout, "value": alt_steps / a_el, "steps": alt_steps,
               "ms_per_step": 1e3 * a_el / alt_steps, "iters": a_res.iters, "algo": a_res.algo,
               "avg_launch_us": a_pass * 1e6,
               "frac": 4.0 * K * d / a_pass / 1e9 / HBM_PEAK_GBS,
               "aggregation_frac": a_passes * 4.0 * K * d / (a_el / alt_steps) / 1e9
               / HBM_PEAK_GBS}
    src = panels if big else X          # the matrix the checks read
    panels = None

    # full-size correctness: the fp64 fixed-point step at the returned aggregate
    check = None
    if not args.no_check and agg_name == "gm2":
        step, gn = fixed_point_step(src, out, allreduce)
        check = {"what": "fp64 gm2 step ||T(g) - g|| at the returned g over the full K x d "
                         "(T = M:174-179); the reference stops at movement <= tol = 1e-5",
                 "fixed_point_step": step, "g_norm": gn, "relative": step / max(gn, 1e-300),
                 "last_movement": res.last_movement, "ok": step <= 1e-4}
    elif not args.no_check:
        check = {"what": "gm (AirComp) never converges (fresh channel draw each iteration, "
                         "SURVEY §3C); parity is pinned by tests/test_gpu_weiszfeld.py",
                 "iters": res.iters, "finite": bool(torch.isfinite(out).all())}

    if rank == 0:
        per_launch_bytes = 4.0 * K * d
        avg_pass_s = (pass_ms / 1e3) / max(launches, 1)
        achieved = per_launch_bytes / avg_pass_s / 1e9
        agg_s = elapsed / args.steps
        agg_frac = passes * per_launch_bytes / agg_s / 1e9 / HBM_PEAK_GBS
        if res.algo in ("gram", "gram_f32"):
            # dominant kernel = the Gram partial: upper-triangle 32x32 tiles of the
            # K-padded Gram, 2 FLOP per MAC, d_local columns.  The scaled-f16 split
            # (gram_kind f16_split) issues 3 f16 MFMAs per tile and 16 columns (hh, hm, mh),
            # the bf16 fallback 4 (hh, hm, mh, mm), gram_f32 one f32 MFMA.  It also reads
            # X once: price both ceilings and report the binding one.
            kt = 1 if K <= 32 else 2 if K <= 64 else 4 if K <= 128 else 8
            split = res.algo == "gram"
            h16 = split and res.gram_kind == "f16_split"
            products = 3 if h16 else 4 if split else 1
            flops = kt * (kt + 1) / 2 * 1024 * 2.0 * d * products
            peak = MFMA_BF16_PEAK_TFLOPS if split else MFMA_F32_PEAK_TFLOPS
            tf = flops / avg_pass_s / 1e12
            gbs = per_launch_bytes / avg_pass_s / 1e9
            kname = "gram_h16_partial" if h16 else "gram_split_partial"
            traffic, traffic_src = pmc_traffic(args.workload, layout, kname) \
                if world == 1 and split else (None, None)
            mf = {"bound": "mfma", "achieved": tf, "peak": peak, "unit": "TFLOP/s",
                  "frac": tf / peak, "traffic": traffic}
            hb = {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                  "frac": gbs / HBM_PEAK_GBS, "traffic": traffic}
            roof, other = (mf, hb) if mf["frac"] >= hb["frac"] else (hb, mf)
            roof.update({"kernel": (f"gram_h16_partial ({layout}; v_mfma_f32_16x16x32_f16, 3 products, "
                                    "scaled h+m split, upper-triangle tiles)") if h16 else
                                   ("gram_split_partial (v_mfma_f32_32x32x16_bf16 x4, h+m split, "
                                    "upper-triangle tiles)") if split else
                                   "gram_partial (v_mfma_f32_32x32x2_f32, upper-triangle tiles)",
                         "gram_kind": res.gram_kind,
                         "traffic_unit": "GB per launch", "traffic_source": traffic_src,
                         "launches_timed": launches, "avg_launch_us": avg_pass_s * 1e6,
                         "algorithmic_flops_per_launch": flops,
                         "algorithmic_bytes_per_launch": per_launch_bytes,
                         "other_ceiling": other,
                         "aggregation_frac": agg_frac,
                         "aggregation_frac_def": "2 reads of X (Gram + closing pass) x 4*K*d_local "
                                                 "/ ms_per_step / 8 TB/s"})
        elif res.algo == "resident":
            # one launch runs the whole aggregation with X held in VGPRs (resident.hip, or
            # for panels the batched kernel with P = 1): X (1.57 MB at C2) is read once, so
            # the kernel is latency-bound — each iteration is a cross-CU exchange of every
            # block's partials plus the phases' VALU work.  Roofline: time per iteration
            # against the exchange floor (the kernel with its compute phases skipped, profiles/)
            us_it = avg_pass_s * 1e6 / max(res.iters, 1)
            # (the floor and the PMC traffic on record are C2's own shape on rows; a panels
            # call of that shape runs the same kernel since round 4 session 2, not quoted)
            fl, fl_src = latency_floor("weiszfeld_resident") if layout == "rows" else (None, None)
            floor = fl["exchange_floor_us_per_iteration"] if fl else None
            traffic, traffic_src = (pmc_traffic(args.workload, layout, "weiszfeld_resident")
                                    if layout == "rows" and world == 1 else (None, None))
            roof = {"bound": "latency", "unit": "us per iteration", "achieved": us_it,
                    "peak": floor, "frac": floor / us_it if floor else None,
                    "frac_def": "exchange floor / achieved time per iteration (<= 1)",
                    "floor_source": fl_src, "traffic": traffic,
                    "traffic_unit": "GB per launch (PMC; X is 4*K*d bytes, read once)",
                    "traffic_source": traffic_src,
                    "kernel": "weiszfeld_resident (every iteration in one launch, X in VGPRs)"
                              if layout == "rows" else "weiszfeld_resident_batched (P = 1)",
                    "launches_timed": launches, "avg_launch_us": avg_pass_s * 1e6,
                    "us_per_iteration": us_it,
                    "streaming_equivalent_frac": agg_frac,
                    "streaming_equivalent_def": "4*K*d*(iters+1) / ms_per_step / 8 TB/s: the bytes "
                                                "the streaming path would move (a comparison, not "
                                                "a roofline: X is read from HBM once per launch)"}
        else:
            traffic, traffic_src = pmc_traffic(args.workload, layout) if world == 1 \
                else (None, None)
            roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "traffic_unit": "GB per launch", "traffic_source": traffic_src,
                    "kernel": f"weiszfeld_pass (STEP, {layout})", "launches_timed": launches,
                    "avg_launch_us": avg_pass_s * 1e6,
                    "algorithmic_bytes_per_launch": per_launch_bytes,
                    "aggregation_frac": agg_frac,
                    "aggregation_frac_def": "4*K*d_local*(iters+1) / ms_per_step / 8 TB/s "
                                            "(BASELINE.md §3)"}
        if dist_path and not args.rehearse_shard and world > 1:
            parallelism = f"d-shard x{world}" + (" (one-GPU gloo rehearsal)" if args.one_gpu else "")
        elif args.rehearse_shard:
            parallelism = (f"rehearsal: rank 0 of a d-shard x{args.rehearse_shard} job on 1 GPU "
                           f"(d_local {d})")
        else:
            parallelism = "d-shard x1 (process group)" if dist_path else "none"
        line = {
            "metric": METRIC,
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
            "config": {"workload": f"{args.workload}: {agg_name} K={K} x d={d_total} fp32, B={B} "
                                   f"Byzantine, tol 1e-5, maxiter {args.maxiter}"
                                   + (f", noise_var {var}" if agg_name == "gm" else ""),
                       "K": K, "d": d_total, "d_local": d, "byzantine": B, "iters": res.iters,
                       "algo": res.algo, "gram_guard": res.guard, "layout": layout,
                       "parallelism": parallelism, "passes_per_aggregation": passes,
                       "input": ("generated straight into the panel layout (no row-major copy "
                                 "resident: it would not fit beside the panels)") if big else
                                "row-major fill, packed to panels once (untimed)"
                                if layout == "panels" else "row-major"},
            "roofline": roof,
            "cpu_baseline": None,
            "check": check,
            "alt_layout": alt,
            "soak": soak,
        }
        if world == 1 and not args.no_cpu and not args.rehearse_shard:
            line["cpu_baseline"] = cpu_baseline(src, g0, agg_name, var, res.iters, d_total,
                                                args.cpu_budget, args.cpu_d)
        print(json.dumps(line), file=json_out, flush=True)
    torch.cuda.synchronize(dev)
    if sg is not None:
        sg.close()                    # RCCL communicator + workspace, before the process group
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
