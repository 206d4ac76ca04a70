# Fresh C4-shard (Gram) and C5 (batched sweep) measurements with the current library.
set -o pipefail
mkdir -p gpurun_out/c4c5
timeout -k 10 300 python -u bench.py --workload c4-shard --no-cpu --steps 10 > gpurun_out/c4c5/c4.json 2> gpurun_out/c4c5/c4.err || { tail -20 gpurun_out/c4c5/c4.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/c4c5/c4.json'));r=d['roofline'];print('c4', d['config']['algo'], round(d['value'],2),'agg/s', r['bound'], round(r['achieved'],1), r['unit'], round(r['frac'],3))"
timeout -k 10 400 python -u tools/sweep_c5.py > gpurun_out/c4c5/c5.jsonl 2> gpurun_out/c4c5/c5.err || { tail -20 gpurun_out/c4c5/c5.err; exit 2; }
cat gpurun_out/c4c5/c5.jsonl
