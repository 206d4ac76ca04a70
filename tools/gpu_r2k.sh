# Round 2: Gram kernel overlap probes on panels (C4 shard, unguarded explicit Gram):
# probe3 = producers convert but store nothing to LDS; probe4 = consumers run MFMAs on
# register fragments (no LDS reads).  Plus the panel tests.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2k
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_panels.py -q --timeout 200 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
export GMAGG_GRAM_UNGUARDED=1
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
for lib in probe3 probe4; do
  GMAGG_LIB=$L/libgmagg_$lib.so step prof_$lib 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$lib -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 5 --warmup 1 --no-cpu --no-check --alt-steps 0
done
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'partial' in r['Name']: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')
"; done
