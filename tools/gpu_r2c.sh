# Round 2: the scaled-f16 Gram kernel — parity tests, C4-shard bench (f16 vs bf16
# split on the same box), rocprof kernel trace of the C4-shard bench.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2c
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step gram_tests 400 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_sharded.py -k "gram" -v -x --timeout 120 --timeout-method thread
step bench_c4 300 python -u bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 0
grep '"metric"' $O/bench_c4.log || true
export GMAGG_GRAM_KIND=bf16; step bench_c4_bf16 300 python -u bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 0 --no-check
grep '"metric"' $O/bench_c4_bf16.log || true
unset GMAGG_GRAM_KIND
cd /tmp && export TMPDIR=/tmp
step prof_c4 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --steps 5 --warmup 1 --no-cpu --no-check --alt-steps 0
find $O/prof_c4 -name "*stats*" | head
