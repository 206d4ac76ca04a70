# Round 2: row-major AirComp gm staged as panels (api.hip): the new parity test, then the
# C3-shape A/B (staged vs GMAGG_STAGE_PANELS=0) on the rows input.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2ao
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_weiszfeld.py -m gpu -q --timeout 200 --timeout-method thread -k "staged or philox or pre_oma" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -ne 0 ] && { grep -E "^FAILED|^E " $O/pytest.log | head -20; exit $rc; }
timeout -k 10 300 python3 tools/rows_bench.py --only a2r > $O/a2r_staged.jsonl 2>&1 || { tail -5 $O/a2r_staged.jsonl; exit 3; }
tail -1 $O/a2r_staged.jsonl
GMAGG_STAGE_PANELS=0 timeout -k 10 300 python3 tools/rows_bench.py --only a2r > $O/a2r_rows.jsonl 2>&1 || { tail -5 $O/a2r_rows.jsonl; exit 4; }
tail -1 $O/a2r_rows.jsonl
