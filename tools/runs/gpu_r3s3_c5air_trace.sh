#!/bin/bash
# kernel trace of the C5 AirComp reading (gm, 1000 iterations per noisy problem) on the
# spill-free batched resident tile
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5air
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5air/prof -o run -- \
  python3 bench.py --workload c5 --reading aircomp --steps 1 --warmup 1 --no-cpu --alt-steps 0 \
  > gpurun_out/c5air/bench.json 2> gpurun_out/c5air/bench.err
