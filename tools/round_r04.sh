# Round measurement set after the f3/OMA kernel rewrite: GPU tests, smoke, bench +
# rocprof + PMC (tools/round_profile.sh), then every per-row timing.
set -o pipefail
bash tools/round_profile.sh r04 || exit $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04/smoke.log 2>&1 || { tail -20 gpurun_out/r04/smoke.log; exit 7; }
timeout -k 10 400 python -u tools/rows_bench.py --out gpurun_out/r04/rows.jsonl > gpurun_out/r04/rows.log 2>&1 || { tail -20 gpurun_out/r04/rows.log; exit 8; }
cat gpurun_out/r04/rows.jsonl
