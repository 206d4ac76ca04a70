# Round 2: resident kernel with fp32 granules + precomputed channel draws: parity
# (weiszfeld + training + sharded + panels suites) and per-phase timing (CPB 1 / 2).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2i
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 400 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_training.py tests/test_gpu_sharded.py -q -x --timeout 200 --timeout-method thread
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
for cpb in 2 1; do
  GMAGG_RES_CPB=$cpb GMAGG_LIB=$L/libgmagg_prof.so step res_$cpb 120 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --no-check
  grep GMK_RES_PROF $O/res_$cpb.log | tail -1
done
step bench_c2 200 python -u bench.py --workload c2 --steps 20 --warmup 3
grep -o '"us_per_iteration": [0-9.]*' $O/bench_c2.log
