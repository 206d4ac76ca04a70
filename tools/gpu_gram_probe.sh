# Timing probes of the split Gram kernel on the C4 shard (results are wrong by design).
set -o pipefail
mkdir -p gpurun_out
for dbg in 0 1 2; do
  GMAGG_GRAM_DEBUG=$dbg timeout -k 10 300 python -u bench.py --workload c4-shard --algo gram --steps 5 --warmup 1 --no-cpu > gpurun_out/r02_probe_$dbg.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r02_probe_$dbg.json'));r=d['roofline'];print('dbg $dbg', round(r['avg_launch_us'],1),'us')"
done
