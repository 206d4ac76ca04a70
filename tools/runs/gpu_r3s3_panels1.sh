#!/bin/bash
# single-call panels -> batched resident kernel (P = 1): the panel / pre-noise tests, then the
# training loop bench on both layouts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_panels.py tests/test_gpu_resident_batched.py \
  "tests/test_gpu_weiszfeld.py::test_pre_oma_equals_oma_then_gm2" > gpurun_out/r3s3_panels1.log 2>&1 &&
timeout -k 10 200 python -u tools/loop_bench.py > gpurun_out/r3s3_loop.jsonl 2>&1
