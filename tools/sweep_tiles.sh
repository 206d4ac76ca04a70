#!/bin/bash
# Sweep streaming-pass tiles (GMAGG_PASS_CFG="NW,LPR,R") per workload; one process per point.
set -o pipefail
out=${1:-gpurun_out/sweep}
mkdir -p "$out"
run() {  # workload cfg
  local wl=$1 cfg=$2 tag
  tag="${wl}_$(echo "$cfg" | tr , _)"
  GMAGG_PASS_CFG=$cfg timeout -k 10 240 python bench.py --workload "$wl" --steps 10 --warmup 2 --no-cpu \
    > "$out/$tag.json" 2> "$out/$tag.err" || { echo "FAILED $tag rc=$?"; return 1; }
  python - "$out/$tag.json" "$wl" "$cfg" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
print(f"{sys.argv[2]:12s} cfg={sys.argv[3]:9s} agg/s={l['value']:8.2f} iters={l['config']['iters']} pass_us={r['avg_launch_us']:8.1f} GB/s={r['achieved']:6.0f} frac={r['frac']:.3f}")
PY
}
for c in 16,8,8 8,8,16 8,4,8 16,4,4 16,4,8; do run c3 $c || exit 1; done
for c in 16,32,8 8,16,8 16,16,4 4,8,8 8,8,8; do run c4-shard $c || exit 1; done
for c in 16,64,4 4,16,4 8,32,4; do run c5-problem $c || exit 1; done
