# Round 2: order-statistic selection with candidate compaction (coordinate.hip).
# f3 parity tests, then rows_bench f3 with the new library and the previous one
# (libgmagg_base.so = HEAD's coordinate.hip), interleaved.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2s
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_other_aggregators.py -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in new base new2; do
  case $v in new*) lib=$L/libgmagg.so;; base*) lib=$L/libgmagg_base.so;; esac
  GMAGG_LIB=$lib timeout -k 10 300 python -u tools/rows_bench.py --only f3 > $O/rows_$v.jsonl 2> $O/rows_$v.err || { tail -20 $O/rows_$v.err; exit 2; }
  echo "== $v"; cut -c1-160 $O/rows_$v.jsonl | grep -v Krum
done
