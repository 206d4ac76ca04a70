# Round 2: same-box A/B of the dead-row-group skip in the panel passes (ab/libgmagg_noskip.so
# = the pass without it, linked from the same objects otherwise); C5 both readings and C3.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2am
mkdir -p $O
cd $GRAFT_REPO_ROOT
for v in skip noskip skip noskip; do
  L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd/libgmagg.so; [ $v = noskip ] && L=$GRAFT_REPO_ROOT/ab/libgmagg_noskip.so
  for r in aircomp prenoise; do
    n=4096; [ $r = aircomp ] && n=1024
    GMAGG_LIB=$L timeout -k 10 200 python3 bench.py --workload c5 --reading $r --problems $n \
      --steps 2 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_${r}_$v.log 2>&1 || { tail -5 $O/c5_${r}_$v.log; exit 3; }
    python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(l['value'],1), round(l['roofline']['achieved'],0), round(l['roofline']['avg_launch_us'],1))" $O/c5_${r}_$v.log $v c5-$r | tee -a $O/summary.txt
  done
  GMAGG_LIB=$L timeout -k 10 200 python3 bench.py --steps 10 --warmup 2 --alt-steps 0 --no-cpu > $O/c3_$v.log 2>&1 || { tail -5 $O/c3_$v.log; exit 4; }
  python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'c3', round(l['value'],2), round(l['roofline']['achieved'],0), round(l['roofline']['avg_launch_us'],1))" $O/c3_$v.log $v | tee -a $O/summary.txt
done
