# A/B of two library builds on the same box, interleaved: C3 bench lines.
#   bash tools/ab_lib.sh [workload] [rounds]
set -o pipefail
mkdir -p gpurun_out
w=${1:-c3}
n=${2:-3}
for i in $(seq 1 $n); do
  for lib in libgmagg.so libgmagg_alt.so; do
    GMAGG_LIB=byzantine_aircomp_amd/$lib timeout -k 10 300 python -u bench.py --workload $w --no-cpu --steps 20 > gpurun_out/ab_$lib.json || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$lib.json'));r=d['roofline'];print('$lib', round(d['value'],3),'agg/s', round(d['ms_per_step'],2),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],4))"
  done
done
