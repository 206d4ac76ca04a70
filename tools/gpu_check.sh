set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01b_pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 gpurun_out/r01b_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/r01b_pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" && \
timeout -k 10 400 python -u bench.py > gpurun_out/r01b_bench.json 2> gpurun_out/r01b_bench.err && cat gpurun_out/r01b_bench.json
