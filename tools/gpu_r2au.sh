# Round 2: staging in d-sharded gm calls: the distributed and staging GPU tests
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2au
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_weiszfeld.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/pytest.log | head -20; exit $rc; }
exit 0
