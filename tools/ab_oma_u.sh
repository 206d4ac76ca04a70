# A/B: OMA Philox kernel with U=2 (default build) vs U=4 groups per step, same box, interleaved.
set -o pipefail
mkdir -p gpurun_out/omau
for r in 1 2; do
  timeout -k 10 200 python -u tools/rows_bench.py --only a4 --out gpurun_out/omau/u2_$r.jsonl > /dev/null || exit 1
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_u4.so timeout -k 10 200 python -u tools/rows_bench.py --only a4 --out gpurun_out/omau/u4_$r.jsonl > /dev/null || exit 2
  python3 -c "import json;a=json.load(open('gpurun_out/omau/u2_$r.jsonl'));b=json.load(open('gpurun_out/omau/u4_$r.jsonl'));print('U=2 %.2f ms  U=4 %.2f ms'%(a['ms'],b['ms']))"
done
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "oma or OMA" 2>&1 | tail -1
