set -o pipefail
O=gpurun_out/r4s1e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_weiszfeld.py -q -x --timeout 200 --timeout-method thread -rf -p no:cacheprovider -k "c4_recipe or guard or gram_split" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
GMAGG_GUARD_DEBUG=1 timeout -k 10 400 python -u bench.py --workload c4 --steps 5 --warmup 1 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 3; }
grep "gram guard" $O/c4.err | tail -2; cut -c1-600 $O/c4.json
for dbg in 0 7; do GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $O/rb_probe_dbg$dbg.log 2>&1 || exit 4; tail -1 $O/rb_probe_dbg$dbg.log; done
GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/c2_exchange_only.json 2> $O/c2x.err || exit 5
timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/c2.json 2> $O/c2.err || exit 6
python -c "
import json
for f in ('c2_exchange_only','c2'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['roofline'].get('us_per_iteration'))"
