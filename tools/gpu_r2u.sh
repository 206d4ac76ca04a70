# Round 2: K=256 STEP / closing-pass tiles on panels (the panel width follows the tile):
# default (16,32,8,1: W=128) vs (8,16,8,2: W=64, two blocks per CU) vs (16,16,4,1: W=64)
# vs (16,64,16,1: W=256).  C4 shard, guarded Gram (AUTO) and streaming, kernel traces.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload c4-shard --steps 10 --warmup 3 --no-cpu --alt-steps 0 --no-check --soak 0"
for cfg in default 8,16,8,2 16,16,4,1 16,64,16,1; do
  for algo in auto stream; do
    n=${cfg//,/_}_$algo
    if [ $cfg = default ]; then unset GMAGG_PASS_CFG; else export GMAGG_PASS_CFG=$cfg; fi
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$n -o run -- python3 $B --algo $algo > $O/$n.log 2>&1
    rc=$?
    echo "== $n rc=$rc $(grep -o '"ms_per_step": [0-9.]*\|"gram_guard": "[a-z]*"\|"algo": "[a-z_0-9]*"' $O/$n.log | tr '\n' ' ')"
    [ $rc -ne 0 ] && { tail -5 $O/$n.log; exit $rc; }
    python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/kt_$n/run_kernel_trace.csv | grep -E "weiszfeld_pass|gram_h16" | cut -c1-110
  done
done
unset GMAGG_PASS_CFG
