# Round 2: batched problems in the panel layout (ProblemPanels): parity, then C5 rows vs panels.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2y
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for lay in panels rows panels rows; do
  timeout -k 10 300 python3 bench.py --workload c5 --no-cpu --soak 0 --layout $lay > $O/c5_$lay.log 2>&1 || { tail -5 $O/c5_$lay.log; exit 2; }
  python3 - $O/c5_$lay.log $lay <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "problems/s %.0f" % d["value"], "ms/sweep %.1f" % d["ms_per_step"], "STEP %.0f GB/s" % r["achieved"],
      "agg_frac %.3f" % r["aggregation_frac"], {k: round(g["problems_per_s"]) for k, g in d["config"]["groups"].items()})
PY
done
