# Round 2: leaner Gram producer: the f16 residual by v_fma_mix (bit check: tools/mixcheck.hip),
# one buffer resource per stage on panels.  Parity (Gram/panel tests), then C4-shard A/B:
# main lib vs libgmagg_nomix (residual by convert-back + subtract) vs libgmagg_noslp
# (no packed f32 FMAs), interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2p
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
hipcc -O3 --offload-arch=gfx950 $GRAFT_REPO_ROOT/tools/mixcheck.hip -o $O/mixcheck > $O/mixcheck_build.log 2>&1 || { echo mixcheck build failed; exit 1; }
step mixcheck 60 $O/mixcheck
step tests 400 python -u -m pytest tests/test_gpu_panels.py tests/test_gpu_weiszfeld.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py -k "gram or panels or Gram or c4" -q -x --timeout 200 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 0"
for v in main nomix noslp main2 nomix2 noslp2; do
  case $v in main*) lib=$L/libgmagg.so;; nomix*) lib=$L/libgmagg_nomix.so;; noslp*) lib=$L/libgmagg_noslp.so;; esac
  GMAGG_LIB=$lib step ab_$v 200 python3 $B
  echo "$v $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*\|"gram_guard": "[a-z]*"' $O/ab_$v.log | tr '\n' ' ')"
done
export GMAGG_GRAM_UNGUARDED=1 GMAGG_GRAM_DEBUG=1
step kt_dbg1 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_dbg1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 3 --warmup 1 --no-cpu --no-check --alt-steps 0
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/kt_dbg1/run_kernel_trace.csv | grep gram_h16 | cut -c1-100
