"""Iteration counts of the GPU paths on the inputs whose count window is undetermined
(tol at or below the fp32 movement floor): the data behind the slacks the tests state."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import byzantine_aircomp_amd as bz  # noqa: E402
from conftest import golden_case  # noqa: E402
import test_gpu_weiszfeld as tw  # noqa: E402

meta, arr = golden_case("gm2_ragged_K7_d777")
X = torch.from_numpy(arr["X"].copy())
o = dict(meta["options"])
if meta.get("guess_supplied"):
    o["guess"] = torch.from_numpy(arr["guess"].copy()).cuda()
print("ragged reference count", meta["iters"])
for algo in ("auto", "stream", "twopass", "resident"):
    try:
        bz.gm2(X.cuda(), dict(o, algo=algo))
        r = bz.aggregators.last_result
        print(f"  ragged rows {algo}: {r.iters} ({r.algo})")
    except Exception as e:  # noqa: BLE001
        print(f"  ragged rows {algo}: {e}")
P = bz.ClientPanels.from_rows(X.cuda())
bz.gm2(P, dict(o))
print("  ragged panels auto:", bz.aggregators.last_result.iters, bz.aggregators.last_result.algo)
for case in tw.GUARD_CASES:
    Xg, p = tw._guard_data(case)
    for algo in ("auto", "stream", "twopass"):
        bz.gm2(Xg.cuda(), {"maxiter": 30, "tol": 1e-5, "guess": p.cuda(), "algo": algo})
        r = bz.aggregators.last_result
        print(f"guard {case} {algo}: {r.iters} ({r.algo}, {r.guard}) last_movement {r.last_movement:.3e}")
    Pg = bz.ClientPanels.from_rows(Xg.cuda())
    bz.gm2(Pg, {"maxiter": 30, "tol": 1e-5, "guess": p.cuda()})
    r = bz.aggregators.last_result
    print(f"guard {case} panels: {r.iters} ({r.algo}, {r.guard}) last_movement {r.last_movement:.3e}")
Xc, g0 = tw._c4_like(256, 1 << 20, seed=4040)
Xc += 0.07
g0 += 0.07
for algo in ("auto", "gram", "stream"):
    bz.gm2(Xc, {"maxiter": 1000, "guess": g0, "algo": algo})
    r = bz.aggregators.last_result
    print(f"c4 floor band {algo}: {r.iters} ({r.algo}, {r.guard}) last_movement {r.last_movement:.3e}")
