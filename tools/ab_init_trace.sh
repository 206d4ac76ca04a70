# INIT plain vs rolling, both under rocprofv3 kernel trace (same box), per-kernel work averages.
set -o pipefail
mkdir -p gpurun_out/initab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in plain roll plain2 roll2; do
  if [ ${v#roll} != $v ]; then export GMAGG_PASS_VARIANT=2; else unset GMAGG_PASS_VARIANT; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/initab/$v -o t -- python bench.py --no-cpu --alt-steps 0 --steps 10 --warmup 2 > gpurun_out/initab/$v.json 2> gpurun_out/initab/$v.err || { tail -5 gpurun_out/initab/$v.err; exit 1; }
  echo "== $v $(python3 -c "import json;d=json.load(open('gpurun_out/initab/$v.json'));print('agg/s %.3f'%d['value'])")"
  python3 tools/trace_summary.py gpurun_out/initab/$v/t_kernel_trace.csv | sed -n 2,3p | cut -c1-120
done
