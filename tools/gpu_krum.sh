# Krum (row f3) retile check: its parity tests, then the f3 timings.
set -o pipefail
mkdir -p gpurun_out/krum
timeout -k 10 300 python -u -m pytest tests/test_gpu_other_aggregators.py -x -q --timeout 120 --timeout-method thread > gpurun_out/krum/pytest.log 2>&1 || { tail -30 gpurun_out/krum/pytest.log; exit 1; }
tail -1 gpurun_out/krum/pytest.log
timeout -k 10 300 python -u tools/rows_bench.py --only f3 --out gpurun_out/krum/rows.jsonl | grep -i krum || exit 2
