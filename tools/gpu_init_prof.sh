# INIT vs STEP pass durations on the C3 panels workload (rocprofv3 kernel trace), per schedule.
set -o pipefail
mkdir -p gpurun_out/initprof
export TMPDIR=/tmp
for v in def 2; do
  if [ $v = def ]; then unset GMAGG_PASS_VARIANT; else export GMAGG_PASS_VARIANT=$v; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/initprof/$v -o c3 -- \
    python bench.py --steps 5 --warmup 1 --no-cpu --alt-steps 0 > gpurun_out/initprof/$v.log 2>&1 || exit 1
  tail -1 gpurun_out/initprof/$v.log | cut -c1-400
  f=$(find gpurun_out/initprof/$v -name 'c3_kernel_trace.csv' | head -1)
  python3 tools/trace_summary.py "$f" | grep -E "calls|weiszfeld" | cut -c1-120
done
unset GMAGG_PASS_VARIANT
