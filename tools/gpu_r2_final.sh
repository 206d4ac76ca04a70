# Round 2 measurement set, part A: the whole GPU suite and smoke() (one process each).
#   gpurun -- bash tools/gpu_r2_final.sh            -> gpurun_out/r2f/{pytest_gpu,smoke}.log
# Part B (PMC passes, bench lines, kernel traces): tools/gpu_r2_final_b.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2f
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 7; }
tail -3 $O/smoke.log
