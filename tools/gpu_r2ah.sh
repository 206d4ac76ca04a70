# Round 2: C5 (panels, fused pre-noise) blocks per problem: GMAGG_BATCH_OVERSUB 2 (default) vs 8 vs 4, interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ah
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in 8 16 32 8 16; do
  GMAGG_BATCH_OVERSUB=$v timeout -k 10 300 python3 bench.py --workload c5 --no-cpu --soak 0 --alt-steps 0 > $O/c5_$v.log 2>&1 || { tail -5 $O/c5_$v.log; exit 2; }
  python3 - $O/c5_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print("oversub", sys.argv[2], "problems/s %.0f" % d["value"], "ms/sweep %.1f" % d["ms_per_step"], "STEP %.0f GB/s" % r["achieved"], "agg_frac %.3f" % r["aggregation_frac"])
PY
done
