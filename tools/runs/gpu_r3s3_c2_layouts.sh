#!/bin/bash
# C2 (AirComp gm, K=50, d=7850, 1000 iterations): rows (C2 single resident kernel) vs panels
# (the batched resident kernel at P = 1), interleaved twice on one box
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python -u bench.py --workload c2 --steps 100 --warmup 5 --alt-steps 0 \
    >> gpurun_out/r3s3_c2_rows.jsonl 2>> gpurun_out/r3s3_c2.err || exit $?
  timeout -k 10 120 python -u bench.py --workload c2 --layout panels --steps 100 --warmup 5 \
    --alt-steps 0 >> gpurun_out/r3s3_c2_panels.jsonl 2>> gpurun_out/r3s3_c2.err || exit $?
done
