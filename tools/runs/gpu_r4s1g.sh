# Round 4 session 1: the closing check (GPU suite, smoke, default bench), then PMC of
# the f3 selection kernels (issue- or latency-bound?).
set -o pipefail
bash tools/final_check.sh || exit $?
O=gpurun_out/r4s1g; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 120 python -u tools/select_bench.py --K 1000 --reps 3 > $O/select.log 2>&1 || exit 5
cat $O/select.log
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_sel -o p -- python3 tools/select_bench.py --K 1000 --reps 1 > $O/pmc_sel.log 2>&1 || exit 6
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sel2 -o p -- python3 tools/select_bench.py --K 1000 --reps 1 > $O/pmc_sel2.log 2>&1 || exit 7
echo pmc-done
