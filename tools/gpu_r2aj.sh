# Round 2: C5 batch size vs the 256 MiB Infinity Cache (a group of B problems is B x 20 MB;
# at B <= 12 every pass after the first could be served on-die).  AirComp reading
# (1000 iterations) and the prenoise reading, 256 and 1024 problems.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2aj
mkdir -p $O
cd $GRAFT_REPO_ROOT
for r in aircomp prenoise; do
  for b in 4 8 12 16 32 1024; do
    n=256; [ $r = prenoise ] && n=4096
    timeout -k 10 200 python3 bench.py --workload c5 --reading $r --problems $n --c5-batch $b \
      --steps 1 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_${r}_b$b.log 2>&1 || { tail -5 $O/c5_${r}_b$b.log; exit 3; }
    python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(l['value'],1), round(l['roofline']['avg_launch_us'],1), {k: round(v['problems_per_s'],1) for k,v in l['config']['groups'].items()})" $O/c5_${r}_b$b.log $r $b | tee -a $O/summary.txt
  done
done
