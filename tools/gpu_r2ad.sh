# Round 2: the coordinate-wise aggregators on ClientPanels; f3 + training GPU tests.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ad
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_other_aggregators.py tests/test_gpu_training.py tests/test_gpu_variance.py -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .*Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/rows_bench.py --only f3 > $O/rows.jsonl 2> $O/rows.err || { tail -20 $O/rows.err; exit 2; }
cut -c1-170 $O/rows.jsonl
