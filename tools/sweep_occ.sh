#!/bin/bash
# Streaming-pass tiles incl. the 2-blocks-per-CU (OCC=2) builds; one process per point.
set -o pipefail
out=${1:-gpurun_out/occ}
mkdir -p "$out"
run() {  # workload cfg
  local tag="${1}_$(echo "$2" | tr , _)"
  GMAGG_PASS_CFG=$2 timeout -k 10 240 python bench.py --workload "$1" --algo stream --steps 10 \
    --warmup 2 --no-cpu > "$out/$tag.json" 2> "$out/$tag.err" || { echo "FAILED $tag rc=$?"; return 1; }
  python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
print(f"{sys.argv[2]:26s} agg/s={l['value']:8.2f} pass_us={r['avg_launch_us']:8.1f} GB/s={r['achieved']:6.0f} frac={r['frac']:.3f}")
PY
}
for c in 16,8,8,1 8,8,16,2 16,8,8,2 16,16,16,1; do run c3 $c || exit 1; done
for c in 16,32,8,1 16,32,8,2; do run c4-shard $c || exit 1; done
for c in 16,64,4,1 16,64,4,2; do run c5-problem $c || exit 1; done
