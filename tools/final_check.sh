# End-of-session check: full GPU suite, smoke, default bench line.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/final/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/final/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" 2>&1 | grep smoke || exit 2
timeout -k 10 400 python -u bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail -20 gpurun_out/final/bench.err; exit 3; }
cat gpurun_out/final/bench.json
