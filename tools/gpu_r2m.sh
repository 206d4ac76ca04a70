# Round 2: INIT pass with the guess on the finisher threads (LDS, by chunk parity) and
# the rolling prefetch; parity on the streaming tests, then C3 A/B under kernel trace:
# new default (rolling INIT) vs GMAGG_PASS_VARIANT=3 (round-1 schedule: plain INIT).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2m
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -2 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step tests 500 python -u -m pytest tests/test_gpu_panels.py tests/test_gpu_weiszfeld.py tests/test_gpu_fullsize.py tests/test_gpu_batched.py -q -x --timeout 200 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
for v in roll plain roll2 plain2; do
  if [ ${v#plain} != $v ]; then export GMAGG_PASS_VARIANT=3; else unset GMAGG_PASS_VARIANT; fi
  step ab_$v 240 rocprofv3 --kernel-trace --output-format csv -d $O/$v -o t -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu --alt-steps 0 --steps 10 --warmup 2
  echo "== $v $(grep -o '"ms_per_step": [0-9.]*' $O/ab_$v.log | head -1)"
  python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/$v/t_kernel_trace.csv | sed -n 2,4p | cut -c1-130
done
