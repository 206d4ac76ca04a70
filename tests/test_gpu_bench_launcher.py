"""`python bench.py --gpus N` as the driver runs it, at N = 2 on the test box's one GPU
(VERDICT r5 item 4): a fresh process that becomes the launcher (no GPU-library call in
it), spawns two ranks (RANK / WORLD_SIZE / MASTER_ADDR 127.0.0.1), each rank running
the d-sharded aggregation (sharded.ShardedGM: the library's sharded host loop, one
all-reduce of the K+2 fp64 partials per iteration) on its half of the columns.  With
`--one-gpu` both ranks share cuda:0 and all-reduce through gloo (RCCL refuses two ranks on
one device); the native RCCL communicator at world > 1 is the driver's 8-GPU run.

Asserted from rank 0's JSON line: n_gpus 2, rank 0's shard of d = 1M is 500,224 columns
(256-aligned), the full-size fixed-point check passes on both ranks' columns, and the
iteration count equals the unsharded call's on the same input (its count window is
[5, 5]: tests/test_gpu_c3_oracle.py)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_bench_two_ranks_c3_small():
    import byzantine_aircomp_amd as bz
    K, d = 1000, 1_000_000
    ctx = bz.context()
    s = torch.cuda.current_stream().cuda_stream
    X = torch.empty(K, d, device="cuda")
    bz._lib.check(ctx.lib.gm_fill_clients_f32(ctx.handle, X.data_ptr(), K, d, d, 200, 0.0, 0.05,
                                              0.25, 0.5, 20211, s), "fill")
    g0 = torch.empty(d, device="cuda")
    bz._lib.check(ctx.lib.gm_fill_normal_f32(ctx.handle, g0.data_ptr(), d, 0.0, 0.01, 20212, s),
                  "fill")
    bz.gm2(bz.ClientPanels.from_rows(X), {"maxiter": 1000, "tol": 1e-5, "guess": g0})
    want_iters = bz.aggregators.last_result.iters
    del X, g0
    torch.cuda.empty_cache()
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-gpu",
                        "--workload", "c3-small", "--steps", "2", "--warmup", "1", "--no-cpu",
                        "--soak", "0", "--alt-steps", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    cfg = line["config"]
    print({k: line[k] for k in ("value", "n_gpus", "ms_per_step")}, cfg["iters"], line["check"])
    assert line["n_gpus"] == 2 and line["steps"] == 2
    assert cfg["d"] == d and cfg["d_local"] == 500_224, cfg
    assert cfg["parallelism"].startswith("d-shard x2"), cfg
    assert line["check"]["ok"], line["check"]
    assert cfg["iters"] == want_iters, (cfg["iters"], want_iters)


@pytest.mark.timeout(600)
def test_bench_two_ranks_c5_sweep():
    """The C5 sweep through the launcher at N = 2: each rank takes its contiguous share of
    every var group (bench.c5_rank_slice), no data-path collective, max-over-ranks timing."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--one-gpu",
                        "--workload", "c5", "--problems", "32", "--steps", "1", "--warmup", "1",
                        "--no-cpu", "--soak", "0", "--alt-steps", "0"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=500)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, p.stdout[-2000:]
    line = json.loads(lines[0])
    cfg = line["config"]
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert cfg["problems"] == 32 and cfg["problems_per_rank"] == 16, cfg
    assert line["check"]["ok"], line["check"]
