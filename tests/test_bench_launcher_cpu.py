"""bench.py's N > 1 plumbing on the CPU: the built-in launcher (`python bench.py --gpus N`
without torchrun) and the C5 problem sharding (the sweep's problems split
over the GPUs, each problem's data and draws independent of N)."""
import json
import os
import subprocess
import sys
import textwrap
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

MOCK = textwrap.dedent("""
    import json, os, sys, time
    r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
    mode = sys.argv[1]
    if mode == "fail" and r == 1:
        sys.exit(3)
    if mode == "fail":
        time.sleep(60)                 # must be stopped by the launcher, not waited for
    if r == 0:
        print("banner line a library printed")
        print(json.dumps({"n_gpus": n, "rank": r, "port": os.environ["MASTER_PORT"],
                          "argv": sys.argv[2:]}))
""")


def _mock(tmp_path):
    p = tmp_path / "mock_rank.py"
    p.write_text(MOCK)
    return str(p)


def test_launcher_relays_rank0_line(tmp_path, capfd):
    rc = bench.launch_ranks(4, [], cmd=[sys.executable, _mock(tmp_path), "ok", "--x"])
    assert rc == 0
    out = capfd.readouterr().out.strip().splitlines()
    assert len(out) == 1                                   # ONE JSON line, the last one
    line = json.loads(out[0])
    assert line["n_gpus"] == 4 and line["rank"] == 0 and line["argv"] == ["--x"]
    assert int(line["port"]) > 0


def test_launcher_fails_fast_when_a_rank_fails(tmp_path, capfd):
    t0 = time.perf_counter()
    rc = bench.launch_ranks(3, [], cmd=[sys.executable, _mock(tmp_path), "fail"])
    assert rc == 3
    assert time.perf_counter() - t0 < 30                   # rank 0 was stopped, not awaited
    assert capfd.readouterr().out == ""


def test_bench_gpus2_without_torchrun_reports_failure_here():
    """No GPU in this container: the launched ranks fail, and `python bench.py --gpus 2
    --one-gpu` must exit non-zero (and promptly) instead of hanging at a barrier."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CUDA_VISIBLE_DEVICES"] = ""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--one-gpu", "--workload", "c3-small", "--steps", "1", "--warmup", "0"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert p.stdout.strip() == ""


@pytest.mark.parametrize("per_var,world", [(1024, 1), (1024, 2), (1024, 8), (1000, 3), (5, 8)])
def test_c5_rank_slices_tile_each_var_group(per_var, world):
    sl = [bench.c5_rank_slice(per_var, world, r) for r in range(world)]
    assert sl[0][0] == 0 and sl[-1][1] == per_var
    assert all(a[1] == b[0] for a, b in zip(sl, sl[1:]))
    sizes = [q1 - q0 for q0, q1 in sl]
    assert max(sizes) - min(sizes) <= 1


def test_c5_keys_do_not_depend_on_the_rank_count():
    """Problem q of var group vi: the same data seed and the same draw key (the batched
    call keys problem p of a call seed + p * SEED_STRIDE) whichever chunk starts at c0."""
    from byzantine_aircomp_amd.batched import SEED_STRIDE
    for vi in range(4):
        base = bench.c5_draw_seed(vi, 0)
        for c0 in (0, 128, 341, 512, 1023):
            for p in (0, 1, 7):
                q = c0 + p
                assert (bench.c5_draw_seed(vi, c0) + p * SEED_STRIDE) % 2 ** 64 == \
                    (base + q * SEED_STRIDE) % 2 ** 64
    seeds = {bench.c5_seed(vi, q) for vi in range(4) for q in range(1024)}
    assert len(seeds) == 4 * 1024                         # every problem its own data
