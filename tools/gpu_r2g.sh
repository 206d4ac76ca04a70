# Round 2: EMNIST / panels training tests; resident-kernel A/B with per-phase
# timing: baseline (CPB 2), no poll back-off, 16 blocks of 4 chunks.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2g
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_training.py -v --timeout 200 --timeout-method thread
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
for v in prof:2 prof_nosleep:2 prof_cpb4:4 prof_cpb4:2; do
  lib=${v%%:*}; cpb=${v##*:}
  GMAGG_RES_CPB=$cpb GMAGG_LIB=$L/libgmagg_$lib.so step res_${lib}_$cpb 120 python -u bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --no-check
  grep GMK_RES_PROF $O/res_${lib}_$cpb.log | tail -1
  grep -o '"us_per_iteration": [0-9.]*' $O/res_${lib}_$cpb.log
done
