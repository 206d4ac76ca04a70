# Round 2: whole GPU suite + smoke after the selection / Philox / K=256 panel-tile changes,
# then the C4-shard bench (guarded Gram on the W=64 panels) and a C3 bench line.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2v
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error" $O/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -3 $O/smoke.log
timeout -k 10 400 python3 bench.py --workload c4-shard --warmup 5 > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 8; }
tail -1 $O/bench_c4.log | cut -c1-400
timeout -k 10 400 python3 bench.py > $O/bench_c3.log 2>&1 || { tail -5 $O/bench_c3.log; exit 9; }
tail -1 $O/bench_c3.log | cut -c1-400
