#!/bin/bash
# A/B the plain (0) and software-pipelined (1) streaming pass on the bench workloads.
set -o pipefail
out=${1:-gpurun_out/ab}
mkdir -p "$out"
for wl in c3 c3-small c4-shard c5-problem; do
  for v in 0 1; do
    GMAGG_PASS_VARIANT=$v timeout -k 10 240 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu \
      > "$out/${wl}_v$v.json" 2> "$out/${wl}_v$v.err" || { echo "FAILED $wl v$v rc=$?"; exit 1; }
    python - "$out/${wl}_v$v.json" "$wl" "$v" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
print(f"{sys.argv[2]:12s} v{sys.argv[3]} agg/s={l['value']:.2f} iters={l['config']['iters']} pass_us={r['avg_launch_us']:.1f} GB/s={r['achieved']:.0f} frac={r['frac']:.3f}")
PY
  done
done
