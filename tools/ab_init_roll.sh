# A/B: INIT pass plain (default) vs rolling prefetch (GMAGG_PASS_VARIANT=2) on the C3 bench.
set -o pipefail
mkdir -p gpurun_out/ab_init
for r in 1 2; do
  for v in default 2; do
    if [ $v = default ]; then unset GMAGG_PASS_VARIANT; else export GMAGG_PASS_VARIANT=$v; fi
    timeout -k 10 200 python -u bench.py --no-cpu --alt-steps 0 --steps 20 > gpurun_out/ab_init/b_${v}_$r.json 2> gpurun_out/ab_init/b_${v}_$r.err || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_init/b_${v}_$r.json'));print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
unset GMAGG_PASS_VARIANT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
GMAGG_PASS_VARIANT=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_init/trace -o roll -- python bench.py --no-cpu --alt-steps 0 --steps 5 --warmup 1 > gpurun_out/ab_init/trace.log 2>&1 || exit 2
python3 tools/trace_summary.py gpurun_out/ab_init/trace/roll_kernel_trace.csv | head -4
