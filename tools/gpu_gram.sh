# Gram split kernel: GPU tests then C4-shard algorithm comparison.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_weiszfeld.py -x -q --timeout 300 --timeout-method thread -k "gram" > gpurun_out/r02_gram_tests.log 2>&1 || { tail -40 gpurun_out/r02_gram_tests.log; exit 1; }
tail -3 gpurun_out/r02_gram_tests.log
for algo in gram gram_f32 stream; do
  timeout -k 10 300 python -u bench.py --workload c4-shard --algo $algo --steps 10 --warmup 2 --no-cpu > gpurun_out/r02_c4_$algo.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r02_c4_$algo.json'));r=d['roofline'];print('$algo', round(d['value'],2),'agg/s', d['config']['iters'], 'iters', r['bound'], round(r['achieved'],1), r['unit'], round(r['frac'],3), 'other', round(r['other_ceiling']['frac'],3) if 'other_ceiling' in r else '')"
done
