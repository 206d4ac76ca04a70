# Round 2: batched row-major AirComp gm staged as panels: the batched GPU tests, then the C5
# AirComp reading on rows, staged vs GMAGG_STAGE_PANELS=0.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ar
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_batched.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/pytest.log | head -20; exit $rc; }
for v in 1 0 1 0; do
  GMAGG_STAGE_PANELS=$v timeout -k 10 200 python3 bench.py --workload c5 --reading aircomp --problems 1024 --layout rows \
    --steps 2 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_rows_stage$v.log 2>&1 || { tail -5 $O/c5_rows_stage$v.log; exit 3; }
  python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('stage', sys.argv[2], round(l['value'],1), round(l['roofline']['achieved'],0), round(l['roofline']['avg_launch_us'],1), {k: round(v['problems_per_s'],1) for k,v in l['config']['groups'].items()})" $O/c5_rows_stage$v.log $v | tee -a $O/summary.txt
done
