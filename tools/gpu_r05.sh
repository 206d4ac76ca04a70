# Full GPU suite, the C3 bench and the P=8 scaling rehearsal.
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r05/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r05/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/r05/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r05/bench.json 2> gpurun_out/r05/bench.err || { tail -20 gpurun_out/r05/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/r05/bench.json'));print('c3', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['alt_layout']['value'])"
for P in 2 8; do
timeout -k 10 200 python -u bench.py --dist --rehearse-shard $P --no-cpu --alt-steps 0 --steps 40 --warmup 3 > gpurun_out/r05/p$P.json 2> gpurun_out/r05/p$P.err || { tail -5 gpurun_out/r05/p$P.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/r05/p$P.json'));print('P=$P', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
