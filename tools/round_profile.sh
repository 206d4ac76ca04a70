#!/bin/bash
# The round's measurement set on one MI355X: GPU tests, the default bench line
# (with CPU baseline), a rocprofv3 kernel-trace summary of the same bench, and the
# two PMC passes (FETCH_SIZE / WRITE_SIZE, one per run) that price HBM traffic.
#   bash tools/round_profile.sh r03 [skip-tests]
set -o pipefail
tag=${1:-r03}
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    > "$out/pytest_gpu.log" 2>&1
  rc=$?; tail -3 "$out/pytest_gpu.log"; [ $rc -gt 1 ] && exit $rc
fi
timeout -k 10 600 python bench.py > "$out/bench.json" 2> "$out/bench.err" || exit 3
tail -1 "$out/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o c3 -- \
  python bench.py --steps 5 --warmup 1 --no-cpu --alt-steps 0 > "$out/trace.log" 2>&1 || exit 4
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/pmc_fetch" -o c3 -- \
  python bench.py --steps 1 --warmup 0 --no-cpu --alt-steps 0 > "$out/pmc_fetch.log" 2>&1 || exit 5
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/pmc_write" -o c3 -- \
  python bench.py --steps 1 --warmup 0 --no-cpu --alt-steps 0 > "$out/pmc_write.log" 2>&1 || exit 6
head -4 "$out/trace/c3_kernel_stats.csv"
