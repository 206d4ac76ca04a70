# Round 2 (session 3, close): rocprofv3 kernel stats of the final C3 and C2 bench runs, and a
# C4-shard bench line with the final code.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ba
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd $R
timeout -k 10 300 python3 bench.py --workload c4-shard > $O/bench_c4.log 2>&1 || { tail -5 $O/bench_c4.log; exit 3; }
tail -1 $O/bench_c4.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o t -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --alt-steps 0 --soak 0 > $O/trace_c3.log 2>&1 || { tail -3 $O/trace_c3.log; exit 4; }
grep '"metric"' $O/trace_c3.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o t -- python3 $R/bench.py --workload c2 --steps 5 --warmup 1 --no-cpu --alt-steps 0 --soak 0 > $O/trace_c2.log 2>&1 || { tail -3 $O/trace_c2.log; exit 5; }
grep '"metric"' $O/trace_c2.log | cut -c1-200
