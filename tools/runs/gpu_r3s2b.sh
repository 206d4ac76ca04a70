set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2b; mkdir -p $o
timeout -k 10 400 python tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant coop= --variant plain=GMAGG_RES_COOP=0 --out $o/ab_c2_coop.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -2 $o/ab.log
GMAGG_RES_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c2plain -o t -- python3 bench.py --workload c2 --no-cpu --soak 0 --alt-steps 0 > $o/c2plain.log 2>&1; echo "c2 plain-launch trace exit $?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/probe_plain -o t -- ./tools/coop_exit_probe plain > $o/probe_plain.log 2>&1; echo "probe plain exit $?"
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/probe_coop -o t -- ./tools/coop_exit_probe coop > $o/probe_coop.log 2>&1; echo "probe coop exit $?"
