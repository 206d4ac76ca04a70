# Round measurement set (session 6: OMA pipelining, rolling row-major passes, Krum retile): GPU tests, smoke, bench +
# rocprof + PMC (tools/round_profile.sh), then every per-row timing.
set -o pipefail
bash tools/round_profile.sh r05 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke.log 2>&1 || { tail -20 gpurun_out/r05/smoke.log; exit 7; }
timeout -k 10 400 python -u tools/rows_bench.py --out gpurun_out/r05/rows.jsonl > gpurun_out/r05/rows.log 2>&1 || { tail -20 gpurun_out/r05/rows.log; exit 8; }
cat gpurun_out/r05/rows.jsonl
