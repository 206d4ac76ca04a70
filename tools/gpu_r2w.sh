# Round 2: batched C5 (gm2 prenoise reading) — blocks per problem (GMAGG_BATCH_OVERSUB) and
# the host poll interval (GMAGG_BATCH_CHECK), C5 bench lines interleaved; batched parity first.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2w
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "2 16" "8 16" "16 16" "8 4" "16 4" "2 16"; do
  set -- $v
  n=os$1_ck$2
  GMAGG_BATCH_OVERSUB=$1 GMAGG_BATCH_CHECK=$2 timeout -k 10 300 python3 bench.py --workload c5 --no-cpu --soak 0 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 2; }
  python3 - $O/$n.log $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "problems/s %.0f" % d["value"], "ms/sweep %.1f" % d["ms_per_step"], "STEP %.0f GB/s" % r["achieved"],
      "launch_us %.0f n %d" % (r["avg_launch_us"], r["launches_timed"]), "agg_frac %.3f" % r["aggregation_frac"],
      {k: round(g["problems_per_s"]) for k, g in d["config"]["groups"].items()})
PY
done
