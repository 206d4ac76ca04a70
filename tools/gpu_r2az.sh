# Round 2 (session 3, final): whole GPU suite + smoke with the final code, then C2, C5 and C3
# bench lines.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2az
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -1 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -2 $O/smoke.log
timeout -k 10 300 python3 bench.py --workload c2 > $O/bench_c2.log 2>&1 || { tail -5 $O/bench_c2.log; exit 8; }
tail -1 $O/bench_c2.log | cut -c1-200
timeout -k 10 300 python3 bench.py --workload c5 > $O/bench_c5.log 2>&1 || { tail -5 $O/bench_c5.log; exit 9; }
tail -1 $O/bench_c5.log | cut -c1-200
timeout -k 10 400 python3 bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 10; }
tail -1 $O/bench_c3.log | cut -c1-200
