# Round 2: Gram producer rows in runs of 8 (row offsets in the load immediate, conflict-free
# ds_writes), panel kernels templated on W; diagonal tiles in 2 MFMA products (hh + h(2m),
# symmetrised in gram_reduce_final).  Parity, then C4-shard A/B: main vs libgmagg_nodiag
# (3 products on diagonal tiles) vs libgmagg_base (317befc), interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2q
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
step tests 400 python -u -m pytest tests/test_gpu_panels.py tests/test_gpu_weiszfeld.py tests/test_gpu_sharded.py tests/test_gpu_fullsize.py tests/test_gpu_distributed.py -k "gram or panels or Gram or c4" -q -x --timeout 200 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 0"
for v in main nodiag base main2 nodiag2 base2; do
  case $v in main*) lib=$L/libgmagg.so;; nodiag*) lib=$L/libgmagg_nodiag.so;; base*) lib=$L/libgmagg_base.so;; esac
  GMAGG_LIB=$lib step ab_$v 200 python3 $B
  echo "$v $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*\|"gram_guard": "[a-z]*"' $O/ab_$v.log | tr '\n' ' ')"
done
export GMAGG_GRAM_UNGUARDED=1 GMAGG_GRAM_DEBUG=1
step kt_dbg1 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_dbg1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 3 --warmup 1 --no-cpu --no-check --alt-steps 0
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/kt_dbg1/run_kernel_trace.csv | grep gram_h16 | cut -c1-100
