set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2q; mkdir -p $o
timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant pf0= --variant pf10=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --variant pf5=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt2.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -3 $o/ab.log
timeout -k 10 300 python -u tools/loop_bench.py > $o/loop.log 2>&1 || { tail -20 $o/loop.log; exit 1; }
tail -8 $o/loop.log
