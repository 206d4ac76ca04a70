# Full GPU check: parity suite, smoke, default bench (C3) and the C4 shard bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/bench_c3.json 2> gpurun_out/bench_c3.err || { tail -20 gpurun_out/bench_c3.err; exit 1; }
cat gpurun_out/bench_c3.json
timeout -k 10 300 python -u bench.py --workload c4-shard --no-cpu --steps 10 > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err || { tail -20 gpurun_out/bench_c4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_c4.json'));r=d['roofline'];print('c4', d['config']['algo'], round(d['value'],2),'agg/s', r['bound'], round(r['achieved'],1), r['unit'], round(r['frac'],3))"
