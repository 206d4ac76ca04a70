# f3 / OMA check on the GPU box: their parity tests, the per-row timings, and a
# kernel-trace summary of the f3 + a4 rows.
set -o pipefail
mkdir -p gpurun_out/f3
timeout -k 10 300 python -u -m pytest tests/test_gpu_other_aggregators.py tests/test_gpu_weiszfeld.py tests/test_gpu_panels.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -k "oma or OMA or aggregat or krum or Krum or median" > gpurun_out/f3/pytest.log 2>&1 || { tail -30 gpurun_out/f3/pytest.log; exit 1; }
tail -1 gpurun_out/f3/pytest.log
timeout -k 10 300 python -u tools/rows_bench.py --out gpurun_out/f3/rows.jsonl --only a4,f3 || exit 1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/f3/prof -o f3 -- python3 tools/rows_bench.py --only a4,f3 > gpurun_out/f3/prof.log 2>&1 || { tail -20 gpurun_out/f3/prof.log; exit 1; }
find gpurun_out/f3/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/f3/kernel_stats.csv
cut -d, -f1-8 gpurun_out/f3/kernel_stats.csv | head -20
