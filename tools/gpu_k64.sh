# K <= 64 tile change: parity suite, C5 sweep, C1/C2 resident timings.
set -o pipefail
mkdir -p gpurun_out/k64
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/k64/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/k64/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/k64/pytest_gpu.log
timeout -k 10 300 python -u tools/sweep_c5.py > gpurun_out/k64/c5.jsonl 2> gpurun_out/k64/c5.err || { tail -20 gpurun_out/k64/c5.err; exit 2; }
cut -c1-200 gpurun_out/k64/c5.jsonl
timeout -k 10 300 python -u tools/rows_bench.py --only c2 --out gpurun_out/k64/rows_c2.jsonl || exit 3
