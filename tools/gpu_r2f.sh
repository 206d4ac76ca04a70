# Round 2: variance + batched OMA tests, C5 sweep bench (prenoise reading, AirComp
# reading as alt, CPU leg), per-phase timing of the resident kernel (GMK_RES_PROF build).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2f
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -3 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_variance.py tests/test_gpu_batched.py tests/test_gpu_training.py -v --timeout 120 --timeout-method thread
for cpb in 1 2; do
  GMAGG_RES_CPB=$cpb GMAGG_LIB=$GRAFT_REPO_ROOT/byzantine_aircomp_amd/libgmagg_prof.so step resprof_$cpb 120 python -u bench.py --workload c2 --steps 2 --warmup 1 --no-cpu --no-check
  grep GMK_RES_PROF $O/resprof_$cpb.log | tail -2
done
step bench_c5 600 python -u bench.py --workload c5 --steps 1 --warmup 1
grep '"metric"' $O/bench_c5.log || true
