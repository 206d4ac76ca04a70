# Round 2: the resident kernel's AirComp coefficients (K <= 64 wave) in fp32 (the reference's
# own precision) instead of fp64: parity tests on the variant (ab/libgmagg_res32.so), then
# the C2 bench, base vs variant alternating on one box.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ay
mkdir -p $O
cd $GRAFT_REPO_ROOT
V=$GRAFT_REPO_ROOT/ab/libgmagg_res32.so
GMAGG_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_training.py -m gpu -q --timeout 200 --timeout-method thread -k "philox or gm_ or loop" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/pytest.log | head -20; exit $rc; }
for v in base res32 base res32 base res32; do
  L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd/libgmagg.so; [ $v = res32 ] && L=$V
  GMAGG_LIB=$L timeout -k 10 200 python3 bench.py --workload c2 --no-cpu --alt-steps 0 > $O/c2_$v.log 2>&1 || { tail -5 $O/c2_$v.log; exit 3; }
  python3 -c "import json,sys; l=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(l['value'],2), round(l['ms_per_step'],3))" $O/c2_$v.log $v | tee -a $O/summary.txt
done
