# Round 2: K = 50 panels tiles with more bytes in flight per CU ((8,32,4) at 3 blocks/CU, (4,32,8)),
# and row groups with no row of the wave skipped (no load issued).
# panel width of ProblemPanels.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2al
mkdir -p $O
cd $GRAFT_REPO_ROOT
for cfg in 8,32,4 8,32,4,3 4,32,8 8,32,4; do
  for r in prenoise aircomp; do
    n=4096; [ $r = aircomp ] && n=1024
    GMAGG_PASS_CFG=$cfg timeout -k 10 200 python3 bench.py --workload c5 --reading $r --problems $n \
      --steps 2 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_${r}_$cfg.log 2>&1 || { tail -5 $O/c5_${r}_$cfg.log; exit 3; }
    python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(l['value'],1), round(l['roofline']['achieved'],0), round(l['roofline']['avg_launch_us'],1), {k: round(v['problems_per_s'],1) for k,v in l['config']['groups'].items()})" $O/c5_${r}_$cfg.log $cfg $r | tee -a $O/summary.txt
  done
done
