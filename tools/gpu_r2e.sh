# Round 2: granule-exchange resident kernel (C1/C2) — GPU parity suite, C2 bench
# (CPB auto, 1, 2), then the full GPU suite.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2e
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step weiszfeld 300 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_training.py tests/test_gpu_batched.py -x -q --timeout 120 --timeout-method thread
for cpb in auto 1 2; do
  if [ $cpb = auto ]; then unset GMAGG_RES_CPB; else export GMAGG_RES_CPB=$cpb; fi
  step bench_c2_$cpb 200 python -u bench.py --workload c2 --steps 20 --warmup 3 --no-cpu
  grep -o '"ms_per_step": [0-9.]*\|"us_per_iteration": [0-9.]*' $O/bench_c2_$cpb.log | tr '\n' ' '; echo
done
unset GMAGG_RES_CPB
step suite 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread
