set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2g; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py > $o/t_resident.log 2>&1 || { tail -30 $o/t_resident.log; exit 1; }
tail -1 $o/t_resident.log
for dbg in 0 1 4; do
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $o/dbg$dbg.log 2>&1 || { tail -5 $o/dbg$dbg.log; exit 1; }
  grep fit $o/dbg$dbg.log
done
timeout -k 10 600 python -u bench.py --workload c5 --no-cpu --alt-steps 0 --soak 0 > $o/c5.json 2> $o/c5.err || { tail -20 $o/c5.err; exit 1; }
python -c "import json;l=json.load(open('$o/c5.json'));print('c5', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['aggregation_frac'], l['check']['ok'], l['config']['groups'])"
