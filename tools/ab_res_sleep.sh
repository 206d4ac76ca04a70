# A/B: resident kernel grid-barrier spin with s_sleep(1) (default) vs no back-off; C1/C2 timings.
set -o pipefail
mkdir -p gpurun_out/ress
for r in 1 2; do
  timeout -k 10 200 python -u tools/rows_bench.py --only c2 --out gpurun_out/ress/s1_$r.jsonl > /dev/null || exit 1
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_s0.so timeout -k 10 200 python -u tools/rows_bench.py --only c2 --out gpurun_out/ress/s0_$r.jsonl > /dev/null || exit 2
  echo "sleep1: $(cut -c1-160 gpurun_out/ress/s1_$r.jsonl | tr '\n' ' ')"
  echo "sleep0: $(cut -c1-160 gpurun_out/ress/s0_$r.jsonl | tr '\n' ' ')"
done
