#!/bin/bash
# resident batched, AirComp draws drawn after the publish + r_k in LDS (no scratch at KR=50
# MODE 1) vs the previous library (libgmagg_alt.so: 352 B/lane of scratch): C2 on panels
# (P = 1), then C5 (gm2, must not move), C5's AirComp reading (gm, 1000 iterations); then the resident-batched GPU tests
set -o pipefail
mkdir -p gpurun_out
L=$PWD/byzantine_aircomp_amd/libgmagg_alt.so
timeout -k 10 300 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--layout,panels,--steps,100,--warmup,5,--alt-steps,0,--no-cpu \
  --variant new= --variant old=GMAGG_LIB=$L --out gpurun_out/r3s3_rb_draws_c2_ab.jsonl > gpurun_out/r3s3_rb_draws_c2_ab.txt 2>&1 &&
timeout -k 10 300 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--no-cpu,--alt-steps,0 \
  --variant new= --variant old=GMAGG_LIB=$L --out gpurun_out/r3s3_rb_draws_c5_ab.jsonl > gpurun_out/r3s3_rb_draws_c5_ab.txt 2>&1 &&
timeout -k 10 400 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--steps,1,--warmup,1,--no-cpu,--alt-steps,0 \
  --variant new= --variant old=GMAGG_LIB=$L --out gpurun_out/r3s3_rb_draws_c5air_ab.jsonl > gpurun_out/r3s3_rb_draws_c5air_ab.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_resident_batched.py tests/test_gpu_panels.py > gpurun_out/r3s3_rb_draws_tests.log 2>&1
