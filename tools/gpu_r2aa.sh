# Round 2: panel tiles of their own at 32 < K <= 64 and 128 < K <= 256: the panel, batched,
# Gram, distributed and training GPU tests, then the C5 bench line (panels by default).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2aa
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_gpu_panels.py tests/test_gpu_batched.py tests/test_gpu_distributed.py tests/test_gpu_training.py tests/test_gpu_sharded.py tests/test_gpu_variance.py -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E  .*Error" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 400 python3 bench.py --workload c5 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 2; }
tail -1 $O/c5.log | cut -c1-300
