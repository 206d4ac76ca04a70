set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2c; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py > $o/t_resident.log 2>&1; rc=$?
tail -5 $o/t_resident.log; grep -E "FAILED|Error|assert" $o/t_resident.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batched.py tests/test_gpu_c5_fullsize.py > $o/t_batched.log 2>&1 || { tail -30 $o/t_batched.log; exit 1; }
tail -2 $o/t_batched.log
timeout -k 10 600 python -u bench.py --workload c5 --no-cpu --alt-steps 0 --soak 0 > $o/c5_res.json 2> $o/c5_res.err || { tail -20 $o/c5_res.err; exit 1; }
python -c "import json;l=json.load(open('$o/c5_res.json'));print('resident c5', l['value'], l['ms_per_step'], l['check'], l['config']['groups'])"
GMAGG_BATCH_RESIDENT=0 timeout -k 10 600 python -u bench.py --workload c5 --no-cpu --alt-steps 0 --soak 0 > $o/c5_stream.json 2> $o/c5_stream.err || { tail -20 $o/c5_stream.err; exit 1; }
python -c "import json;l=json.load(open('$o/c5_stream.json'));print('stream c5', l['value'], l['ms_per_step'])"
