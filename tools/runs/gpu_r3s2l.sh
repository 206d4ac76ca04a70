set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2l; mkdir -p $o
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_batched.py tests/test_gpu_c5_fullsize.py > $o/t.log 2>&1; rc=$?
tail -3 $o/t.log; grep -E "^FAILED|Error" $o/t.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u bench.py --workload c5 --no-cpu --soak 0 > $o/c5.json 2> $o/c5.err || { tail -20 $o/c5.err; exit 1; }
python -c "import json;l=json.load(open('$o/c5.json'));print('c5', l['value'], json.dumps(l['alt_layout']))"
