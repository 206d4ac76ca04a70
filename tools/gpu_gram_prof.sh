# C4-shard Gram variants: bench lines + rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_weiszfeld.py -x -q --timeout 300 --timeout-method thread -k gram > gpurun_out/r02_gram_tests.log 2>&1 || { tail -40 gpurun_out/r02_gram_tests.log; exit 1; }
tail -2 gpurun_out/r02_gram_tests.log
for algo in gram gram_f32; do
  timeout -k 10 300 python -u bench.py --workload c4-shard --algo $algo --steps 10 --warmup 2 --no-cpu > gpurun_out/r02_c4_$algo.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r02_c4_$algo.json'));r=d['roofline'];print('$algo', round(d['value'],2),'agg/s', d['config']['iters'], 'iters', r['bound'], round(r['achieved'],1), r['unit'], round(r['frac'],3), 'us', round(r['avg_launch_us'],1))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4gram -o c4gram -- python3 bench.py --workload c4-shard --algo gram --steps 5 --warmup 1 --no-cpu > gpurun_out/r02_prof_c4gram.log 2>&1 || { tail -20 gpurun_out/r02_prof_c4gram.log; exit 1; }
find gpurun_out/prof_c4gram -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-8 {} | head -12'
