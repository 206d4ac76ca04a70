# Round 2: C3 row-major (the drop-in [K, d] input) STEP tile sweep at K=1000.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ac
mkdir -p $O
cd $GRAFT_REPO_ROOT
for cfg in 8,8,16,2 16,8,8,1 16,8,8,2 16,16,16,1 16,4,4,1 8,8,16,2; do
  GMAGG_PASS_CFG=$cfg timeout -k 10 300 python3 bench.py --layout rows --algo stream --steps 5 --warmup 1 --no-cpu --no-check --soak 0 --alt-steps 0 > $O/rows_$cfg.log 2>&1 || { echo "$cfg failed"; tail -3 $O/rows_$cfg.log; continue; }
  python3 - $O/rows_$cfg.log $cfg <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "agg/s %.2f" % d["value"], "STEP us %.0f" % r["avg_launch_us"], "frac %.3f" % r["frac"], "agg_frac %.3f" % r["aggregation_frac"])
PY
done
