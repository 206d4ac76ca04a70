# Rolling prefetch as the default for row-major STEP passes: parity suite, C3 (panels +
# row-major alt layout), C5 sweep.
set -o pipefail
mkdir -p gpurun_out/rr
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/rr/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/rr/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/rr/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu --alt-steps 10 > gpurun_out/rr/bench.json 2> gpurun_out/rr/bench.err || { tail -20 gpurun_out/rr/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('gpurun_out/rr/bench.json'));a=d['alt_layout'];print('c3 panels', d['value'], d['roofline']['avg_launch_us'], 'rows', a['value'], a['avg_launch_us'])"
GMAGG_PASS_VARIANT=0 timeout -k 10 300 python -u bench.py --no-cpu --alt-steps 10 --layout rows > gpurun_out/rr/bench_rows_plain.json 2> gpurun_out/rr/bench_rows_plain.err || { tail -20 gpurun_out/rr/bench_rows_plain.err; exit 3; }
python3 -c "import json;d=json.load(open('gpurun_out/rr/bench_rows_plain.json'));print('c3 rows plain', d['value'], d['roofline']['avg_launch_us'])"
timeout -k 10 300 python -u tools/sweep_c5.py > gpurun_out/rr/c5.jsonl 2> gpurun_out/rr/c5.err || { tail -20 gpurun_out/rr/c5.err; exit 4; }
tail -1 gpurun_out/rr/c5.jsonl
