# Round 2: batched-grid rounds (GMAGG_BATCH_OVERSUB) for the C5 AirComp reading, where every
# problem runs all 1000 iterations (no early finishers to spread), vs the prenoise reading.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2an
mkdir -p $O
cd $GRAFT_REPO_ROOT
for ov in 1 2 4 8 1 8; do
  for r in aircomp prenoise; do
    n=4096; [ $r = aircomp ] && n=1024
    GMAGG_BATCH_OVERSUB=$ov timeout -k 10 200 python3 bench.py --workload c5 --reading $r --problems $n \
      --steps 2 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_${r}_$ov.log 2>&1 || { tail -5 $O/c5_${r}_$ov.log; exit 3; }
    python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(l['value'],1), round(l['roofline']['achieved'],0), round(l['roofline']['avg_launch_us'],1), {k: round(v['problems_per_s'],1) for k,v in l['config']['groups'].items()})" $O/c5_${r}_$ov.log $ov $r | tee -a $O/summary.txt
  done
done
