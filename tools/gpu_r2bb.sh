# Round 2: nontemporal write-back in the fused OMA + INIT pass (ab/libgmagg_ntst.so) vs the
# plain float4 store: pre_oma parity on the variant, then C5 (prenoise) alternating on one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2bb
mkdir -p $O
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ab/libgmagg_ntst.so
GMAGG_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_batched.py -m gpu -q --timeout 200 --timeout-method thread -k "pre_oma or prenoise or panels_match" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/pytest.log | head -20; exit $rc; }
for v in base ntst base ntst base ntst; do
  L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd/libgmagg.so; [ $v = ntst ] && L=$V
  GMAGG_LIB=$L timeout -k 10 200 python3 bench.py --workload c5 --steps 3 --warmup 1 --alt-steps 0 --no-cpu > $O/c5_$v.log 2>&1 || { tail -5 $O/c5_$v.log; exit 3; }
  python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],1), round(l['ms_per_step'],2), round(l['roofline']['achieved'],0), {k: round(v['problems_per_s'],1) for k,v in l['config']['groups'].items()})" $O/c5_$v.log $v | tee -a $O/summary.txt
done
