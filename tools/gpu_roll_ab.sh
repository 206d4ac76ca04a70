# A/B of the pass schedules on the C3 panels workload, interleaved in one call:
# GMAGG_PASS_VARIANT unset (panels: rolling STEP + plain INIT), 2 (rolling everywhere), 0 (plain).
set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3; do
  for v in def 2 0; do
    if [ $v = def ]; then unset GMAGG_PASS_VARIANT; else export GMAGG_PASS_VARIANT=$v; fi
    timeout -k 10 300 python -u bench.py --workload c3 --no-cpu --steps 10 --warmup 2 --alt-steps 0 > gpurun_out/roll_$v.json || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/roll_$v.json'));r=d['roofline'];print('v=$v', round(d['value'],3),'agg/s', round(d['ms_per_step'],2),'ms STEP', round(r['avg_launch_us'],1),'us', round(r['frac'],4))"
  done
done
unset GMAGG_PASS_VARIANT
