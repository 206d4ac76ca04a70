# Round 2: OMA pre-noise fused into the INIT pass (MODE 4): parity (fused == OMA then gm2,
# single and batched, rows and panels, every fallback path), OMA / batched / panel tests,
# then C5 fused vs separate OMA, interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_batched.py tests/test_gpu_panels.py -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .*Error" $O/pytest.log | head -20; exit $rc; }
for v in fused sep fused sep; do
  f=""; [ $v = sep ] && f="--separate-oma"
  timeout -k 10 300 python3 bench.py --workload c5 --no-cpu --soak 0 $f > $O/c5_$v.log 2>&1 || { tail -5 $O/c5_$v.log; exit 2; }
  python3 - $O/c5_$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "problems/s %.0f" % d["value"], "ms/sweep %.1f" % d["ms_per_step"], "STEP %.0f GB/s" % r["achieved"],
      "agg_frac %.3f" % r["aggregation_frac"], {k: round(g["problems_per_s"]) for k, g in d["config"]["groups"].items()})
PY
done
