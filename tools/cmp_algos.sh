#!/bin/bash
# Compare streaming vs Gram (and anything else) per workload: one bench process per point.
#   bash tools/cmp_algos.sh OUTDIR "c4-shard c5-problem c3-small" "stream gram"
set -o pipefail
out=${1:-gpurun_out/cmp}
wls=${2:-"c4-shard c5-problem c3-small"}
algos=${3:-"stream gram"}
mkdir -p "$out"
for wl in $wls; do
  for al in $algos; do
    f="$out/${wl}_${al}.json"
    timeout -k 10 240 python bench.py --workload "$wl" --algo "$al" --steps 10 --warmup 2 --no-cpu \
      > "$f" 2> "$out/${wl}_${al}.err" || { echo "FAILED $wl $al rc=$?"; exit 1; }
    python - "$f" "$wl" "$al" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = l["roofline"]
print(f"{sys.argv[2]:12s} {sys.argv[3]:8s} agg/s={l['value']:9.2f} ms={l['ms_per_step']:8.3f} "
      f"iters={l['config']['iters']} main_kernel_us={r['avg_launch_us']:8.1f}")
PY
  done
done
