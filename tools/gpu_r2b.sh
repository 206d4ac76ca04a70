# Round 2 (session b): the sharded-Gram failure with the guard's numbers printed,
# then C4-shard and C2 bench lines (with CPU legs) and a C4 kernel-trace baseline.
set -o pipefail
O=gpurun_out/r2b
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
export GMAGG_GUARD_DEBUG=1
step gram_shard 300 python -u -m pytest tests/test_gpu_sharded.py -k gram -v -s --timeout 200 --timeout-method thread
unset GMAGG_GUARD_DEBUG
step bench_c4 300 python -u bench.py --workload c4-shard --steps 10 --warmup 2
grep '"metric"' $O/bench_c4.log || true
step bench_c2 300 python -u bench.py --workload c2 --steps 10 --warmup 2
grep '"metric"' $O/bench_c2.log || true
cd /tmp && export TMPDIR=/tmp
step prof_c4 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --steps 5 --warmup 1 --no-cpu --no-check --alt-steps 0
