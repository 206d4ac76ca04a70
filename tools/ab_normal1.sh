# A/B: AirComp column noise with the hardware Box-Muller (default) vs the precise one
# (GMK_NORMAL1_PRECISE build), a2 STEP pass at the C3 shape, same box, interleaved.
set -o pipefail
mkdir -p gpurun_out/n1
for r in 1 2; do
  timeout -k 10 200 python -u tools/rows_bench.py --only a2 --out gpurun_out/n1/hw_$r.jsonl > /dev/null || exit 1
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_np.so timeout -k 10 200 python -u tools/rows_bench.py --only a2 --out gpurun_out/n1/precise_$r.jsonl > /dev/null || exit 2
  python3 -c "import json;a=json.load(open('gpurun_out/n1/hw_$r.jsonl'));b=json.load(open('gpurun_out/n1/precise_$r.jsonl'));print('hw %.1f us  precise %.1f us'%(a['pass_us'],b['pass_us']))"
done
