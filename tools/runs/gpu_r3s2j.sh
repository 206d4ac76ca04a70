set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2j; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_c5_fullsize.py > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 300 python -u tools/rb_probe.py --quick > $o/probe_cur.log 2>&1 || { tail -5 $o/probe_cur.log; exit 1; }
grep fit $o/probe_cur.log
timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant cur= --variant old=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -2 $o/ab.log
