# Round 2: where the C5 sweep's time goes (kernel trace of one timed sweep, prenoise reading).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2x
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_c5 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 1 --warmup 1 --no-cpu --soak 0 --alt-steps 0 > $O/c5.log 2>&1 || { tail -5 $O/c5.log; exit 1; }
tail -1 $O/c5.log | cut -c1-200
python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/kt_c5/run_kernel_trace.csv | head -14 | cut -c1-150
