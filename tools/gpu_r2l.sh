# Round 2: lean Gram producer (block-uniform scale, one FMA per element, immediate LDS
# offsets, compile-time panel addressing): parity, C4-shard bench, probes 0/1/2 on panels.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2l
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest tests/test_gpu_panels.py tests/test_gpu_weiszfeld.py tests/test_gpu_distributed.py tests/test_gpu_sharded.py -k "gram or panels or Gram" -q -x --timeout 200 --timeout-method thread
step bench_c4 300 python -u bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 5
grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*\|"layout": "[a-z]*"' $O/bench_c4.log | tr '\n' ' '; echo
cd /tmp && export TMPDIR=/tmp
export GMAGG_GRAM_UNGUARDED=1
for dbg in 0 1 2; do
  export GMAGG_GRAM_DEBUG=$dbg
  step prof_dbg$dbg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dbg$dbg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 5 --warmup 1 --no-cpu --no-check --alt-steps 0
done
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'partial' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"; done
