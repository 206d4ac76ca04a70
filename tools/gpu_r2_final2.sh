# Round 2 measurement set (session 3), part B: for the C3 (default) and C4-shard workloads, the two
# PMC passes (FETCH_SIZE, WRITE_SIZE: one per run) summarised into profiles/ (which the
# bench reads for its "traffic" field), then the bench lines (C3 and C4 with their CPU
# baselines, C2, C5) and a kernel trace of each of C3 and C4.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2g
R=$GRAFT_REPO_ROOT
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 $O/$name.log | cut -c1-300
  if [ $rc -ne 0 ]; then exit $rc; fi
}
cd /tmp && export TMPDIR=/tmp
for w in c3 c4-shard; do
  case $w in c3) lay=panels;; c4-shard) lay=panels;; esac
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch_$w -o p -- python3 $R/bench.py --workload $w --steps 1 --warmup 0 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/pmc_fetch_$w.log 2>&1 || { echo "pmc fetch $w failed"; tail -3 $O/pmc_fetch_$w.log; exit 5; }
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write_$w -o p -- python3 $R/bench.py --workload $w --steps 1 --warmup 0 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/pmc_write_$w.log 2>&1 || { echo "pmc write $w failed"; tail -3 $O/pmc_write_$w.log; exit 6; }
  python3 $R/tools/pmc_summary.py $O/pmc_fetch_$w/p_counter_collection.csv $O/pmc_write_$w/p_counter_collection.csv $O/r2b_pmc_${w}_$lay.json "$w $lay" > $O/pmc_summary_$w.log 2>&1 || { cat $O/pmc_summary_$w.log; exit 8; }
  cp $O/r2b_pmc_${w}_$lay.json $R/profiles/
done
step bench_c3 600 python3 $R/bench.py
step bench_c4 600 python3 $R/bench.py --workload c4-shard --warmup 5
step bench_c2 300 python3 $R/bench.py --workload c2
step bench_c5 400 python3 $R/bench.py --workload c5
step trace_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c3 -o t -- python3 $R/bench.py --steps 5 --warmup 1 --no-cpu --alt-steps 0 --soak 0
step trace_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o t -- python3 $R/bench.py --workload c4-shard --steps 5 --warmup 1 --no-cpu --alt-steps 0 --soak 0
python3 $R/tools/trace_summary.py $O/trace_c3/t_kernel_trace.csv $O/r2b_kernel_trace_c3_panels.txt | sed -n 1,5p | cut -c1-150
python3 $R/tools/trace_summary.py $O/trace_c4/t_kernel_trace.csv $O/r2b_kernel_trace_c4_shard_panels.txt | sed -n 1,8p | cut -c1-150
