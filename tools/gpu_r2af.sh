# Round 2: resident kernel draws the column noise of the next pass right after publishing
# (off the critical path).  Resident / gm parity tests, then C2 new vs base interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2af
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_training.py -q --timeout 200 --timeout-method thread -k "resident or gm_ or philox or Philox or loop or C2 or c2" > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -gt 1 ] && exit $rc; [ $rc -eq 1 ] && { grep -E "^FAILED" $O/pytest.log | head; exit 1; }
for v in new base new2 base2; do
  case $v in new*) lib=$L/libgmagg.so;; base*) lib=$L/libgmagg_base.so;; esac
  GMAGG_LIB=$lib timeout -k 10 200 python3 bench.py --workload c2 --no-cpu --soak 0 --steps 40 > $O/c2_$v.log 2>&1 || { tail -5 $O/c2_$v.log; exit 2; }
  echo "$v $(grep -o '"ms_per_step": [0-9.]*\|"us_per_iteration": [0-9.]*' $O/c2_$v.log | tr '\n' ' ')"
done
