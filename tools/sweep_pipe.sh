#!/bin/bash
# A/B plain vs software-pipelined streaming pass per tile (one process per point).
#   GMAGG_PASS_VARIANT: 0 plain, 1 pipelined;  GMAGG_PASS_CFG="NW,LPR,R"
set -o pipefail
out=${1:-gpurun_out/pipe}
mkdir -p "$out"
run() {  # workload variant cfg
  local tag="${1}_v${2}_$(echo "$3" | tr , _)"
  GMAGG_PASS_VARIANT=$2 GMAGG_PASS_CFG=$3 timeout -k 10 240 python bench.py --workload "$1" \
    --algo stream --steps 10 --warmup 2 --no-cpu > "$out/$tag.json" 2> "$out/$tag.err" \
    || { echo "FAILED $tag rc=$?"; return 1; }
  python - "$out/$tag.json" "$tag" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
print(f"{sys.argv[2]:28s} agg/s={l['value']:8.2f} pass_us={r['avg_launch_us']:8.1f} GB/s={r['achieved']:6.0f} frac={r['frac']:.3f}")
PY
}
run c3 0 16,8,8 || exit 1
run c3 0 8,8,16 || exit 1
run c3 1 8,8,16 || exit 1
run c3-small 0 16,8,8 || exit 1
run c3-small 1 8,8,16 || exit 1
run c4-shard 0 16,32,8 || exit 1
run c4-shard 1 8,16,8 || exit 1
run c4-shard 1 8,32,4 || exit 1
