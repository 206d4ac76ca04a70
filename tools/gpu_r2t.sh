# Round 2: Philox rounds on v_bitop3_b32 (philox.h).  Philox-dependent parity tests, then
# OMA (a4) and the C2 resident loop with the new library and the previous one.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2t
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_weiszfeld.py tests/test_gpu_batched.py tests/test_gpu_sharded.py -x -q --timeout 120 --timeout-method thread -k "philox or Philox or oma or OMA or gm_ or resident or batched" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new base new2 base2; do
  case $v in new*) lib=$L/libgmagg.so;; base*) lib=$L/libgmagg_base.so;; esac
  GMAGG_LIB=$lib timeout -k 10 300 python -u tools/rows_bench.py --only a4,c2 > $O/rows_$v.jsonl 2> $O/rows_$v.err || { tail -20 $O/rows_$v.err; exit 2; }
  echo "== $v"; cut -c1-200 $O/rows_$v.jsonl
done
