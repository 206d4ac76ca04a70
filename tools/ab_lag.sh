set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for v in lag nolag; do
  if [ $v = nolag ]; then export GMAGG_NO_LAG=1; else unset GMAGG_NO_LAG; fi
  timeout -k 10 300 python -u bench.py --no-cpu --steps 20 > gpurun_out/ab_$v.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));r=d['roofline'];print('$v', round(d['value'],3),'agg/s', round(d['ms_per_step'],2),'ms', r['launches_timed'], round(r['avg_launch_us'],1),'us', round(r['frac'],4))"
done
done
