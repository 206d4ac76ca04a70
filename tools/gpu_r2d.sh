# Round 2: f16 Gram fix check + per-kernel timing probes (rocprof stats) of the
# C4-shard Gram: full kernel, consumers without MFMAs (1), producers without loads (2).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2d
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step gram_tests 400 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -k "gram" -v --timeout 200 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
export GMAGG_GRAM_UNGUARDED=1
for dbg in 0 1 2; do
  export GMAGG_GRAM_DEBUG=$dbg
  step prof_dbg$dbg 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_dbg$dbg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 5 --warmup 1 --no-cpu --no-check --alt-steps 0
done
unset GMAGG_GRAM_DEBUG
export GMAGG_GRAM_KIND=bf16
step prof_bf16 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bf16 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 5 --warmup 1 --no-cpu --no-check --alt-steps 0
for f in $(find $O -name "*kernel_stats.csv"); do echo "== $f"; cut -d, -f1-4 $f | grep -i "gram\|Name" | head -5; done
