set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2o; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_training.py tests/test_gpu_resident_batched.py > $o/t.log 2>&1 || { tail -30 $o/t.log; exit 1; }
tail -1 $o/t.log
timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant fast= --variant prev=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c2.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; exit 1; }
tail -2 $o/ab.log
