# Round 2: resident kernel (block-reduced movement partials, poll-one-granule)
# parity + per-phase A/B (poll1 vs poll0, CPB 1 / 2).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2h
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_training.py -q -x --timeout 200 --timeout-method thread
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
for v in prof:2 prof_poll0:2 prof:1 prof_poll0:1; do
  lib=${v%%:*}; cpb=${v##*:}
  GMAGG_RES_CPB=$cpb GMAGG_LIB=$L/libgmagg_$lib.so step res_${lib}_$cpb 120 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --no-check
  grep GMK_RES_PROF $O/res_${lib}_$cpb.log | tail -1
  grep -o '"us_per_iteration": [0-9.]*' $O/res_${lib}_$cpb.log
done
step bench_c2 200 python -u bench.py --workload c2 --steps 20 --warmup 3
grep -o '"us_per_iteration": [0-9.]*' $O/bench_c2.log
# alloca-to-LDS promotion A/B (the same sources built with -mllvm -disable-promote-alloca-to-lds)
for lib in libgmagg libgmagg_np; do
  GMAGG_LIB=$L/$lib.so step c3_$lib 300 python -u bench.py --steps 10 --warmup 2 --no-cpu --alt-steps 3
  grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $O/c3_$lib.log | tr '\n' ' '; echo
  GMAGG_LIB=$L/$lib.so step c4_$lib 300 python -u bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 0 --no-check
  grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $O/c4_$lib.log | tr '\n' ' '; echo
done
