# Panel-layout check on one MI355X: the panel parity tests, then C3 bench lines
# rows vs panels, plain vs rolling-prefetch schedule, interleaved.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_panels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_panels.log 2>&1 || { echo PYTEST_FAIL; tail -40 gpurun_out/pytest_panels.log; exit 1; }
tail -1 gpurun_out/pytest_panels.log
for r in 1 2; do
  for lay in rows panels; do
    for v in 0 2; do
      GMAGG_PASS_VARIANT=$v timeout -k 10 300 python -u bench.py --workload c3 --layout $lay --no-cpu --steps 10 --warmup 2 > gpurun_out/pan_${lay}_$v.json || exit 1
      python3 -c "import json;d=json.load(open('gpurun_out/pan_${lay}_$v.json'));r=d['roofline'];print('$lay v$v', round(d['value'],3),'agg/s', round(d['ms_per_step'],2),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],4))"
    done
  done
done
