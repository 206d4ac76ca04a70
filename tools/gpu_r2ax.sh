# Round 2: batched calls with lagged done-count polls + an adaptive grid (blocks per
# problem from the problems left): batched GPU tests, then C5 A/B on one box:
# new (default) vs lagged polls only (GMAGG_BATCH_ADAPT=0) vs the old synchronous poll
# every 16 iterations (GMAGG_BATCH_CHECK=16).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ax
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py tests/test_gpu_weiszfeld.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/pytest.log | head -20; exit $rc; }
run() {  # name env...
  n=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --workload c5 --steps 3 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_$n.log 2>&1 || { tail -5 $O/c5_$n.log; return 1; }
  python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), round(l['roofline']['achieved'],0), round(l['roofline']['avg_launch_us'],1), l['roofline']['launches_timed'], {k: round(v['problems_per_s'],1) for k,v in l['config']['groups'].items()})" $O/c5_$n.log $n | tee -a $O/summary.txt
}
run new GMAGG_X=1 && run lag_only GMAGG_BATCH_ADAPT=0 && run old GMAGG_BATCH_CHECK=16 && \
run new2 GMAGG_X=1 && run lag_only2 GMAGG_BATCH_ADAPT=0 && run old2 GMAGG_BATCH_CHECK=16
