# Quick GPU check: parity suite, then the C3 and C4-shard bench lines (no CPU leg).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for w in c3 c4-shard; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu --steps 20 > gpurun_out/q_$w.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/q_$w.json'));r=d['roofline'];print('$w', d['config']['algo'], round(d['value'],3),'agg/s', round(d['ms_per_step'],2),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],4))"
done
