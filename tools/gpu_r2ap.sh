# Round 2: HBM traffic of the batched C5 STEP pass (rocprofv3 FETCH_SIZE / WRITE_SIZE, one
# counter per pass) on the AirComp reading, where every launch covers all 1024 problems of
# a group: per-launch traffic vs 1024 x 4Kd algorithmic bytes.  Then a C5 kernel trace.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ap
R=$GRAFT_REPO_ROOT
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
A="--workload c5 --reading aircomp --problems 4096 --steps 1 --warmup 0 --no-cpu --alt-steps 0"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o p -- python3 $R/bench.py $A > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -3 $O/pmc_fetch.log; exit 5; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o p -- python3 $R/bench.py $A > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -3 $O/pmc_write.log; exit 6; }
python3 $R/tools/pmc_summary.py $O/pmc_fetch/p_counter_collection.csv $O/pmc_write/p_counter_collection.csv $O/r2c_pmc_c5_panels.json "c5 aircomp panels" > $O/pmc_summary.log 2>&1 || { cat $O/pmc_summary.log; exit 8; }
cat $O/pmc_summary.log | head -20
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c5 -o t -- python3 $R/bench.py --workload c5 --steps 2 --warmup 1 --no-cpu --alt-steps 0 > $O/trace_c5.log 2>&1 || { tail -3 $O/trace_c5.log; exit 9; }
tail -1 $O/trace_c5.log | cut -c1-200
