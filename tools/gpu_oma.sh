# OMA (row a4) check on the GPU box: every OMA parity test, then the C3-size timing.
set -o pipefail
mkdir -p gpurun_out/oma
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "oma or OMA" > gpurun_out/oma/pytest.log 2>&1 || { tail -30 gpurun_out/oma/pytest.log; exit 1; }
tail -1 gpurun_out/oma/pytest.log
timeout -k 10 300 python -u tools/rows_bench.py --only a4 --out gpurun_out/oma/rows.jsonl || exit 1
