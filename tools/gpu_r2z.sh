# Round 2: C5 on ProblemPanels, K=50 tile sweep (the panel width follows the tile).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2z
mkdir -p $O
cd $GRAFT_REPO_ROOT
for cfg in default 8,32,4 4,16,4 8,32,4 default; do
  if [ $cfg = default ]; then unset GMAGG_PASS_CFG; else export GMAGG_PASS_CFG=$cfg; fi
  timeout -k 10 300 python3 bench.py --workload c5 --no-cpu --soak 0 --layout panels > $O/c5_$cfg.log 2>&1 || { tail -5 $O/c5_$cfg.log; exit 2; }
  python3 - $O/c5_$cfg.log $cfg <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "problems/s %.0f" % d["value"], "ms/sweep %.1f" % d["ms_per_step"], "STEP %.0f GB/s" % r["achieved"],
      "agg_frac %.3f" % r["aggregation_frac"], {k: round(g["problems_per_s"]) for k, g in d["config"]["groups"].items()})
PY
done
