# Per-rank time of the N = 2/4/8 strong-scaling C3 job, rehearsed on one GPU: rank 0's
# d-shard with its per-iteration exchange over a 1-rank RCCL communicator.
set -o pipefail
mkdir -p gpurun_out/scal
for P in 1 2 4 8; do
  if [ $P = 1 ]; then extra=""; else extra="--rehearse-shard $P"; fi
  timeout -k 10 200 python -u bench.py --dist $extra --no-cpu --alt-steps 0 --steps 40 --warmup 3 > gpurun_out/scal/p$P.json 2> gpurun_out/scal/p$P.err || { tail -5 gpurun_out/scal/p$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/scal/p$P.json'));r=d['roofline'];print('P=$P', round(d['value'],2), 'agg/s', round(d['ms_per_step'],3), 'ms', 'iters', d['config']['iters'], 'pass_us', round(r['avg_launch_us'],1), 'frac', round(r['frac'],3))"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/scal/trace8 -o p8 -- python bench.py --dist --rehearse-shard 8 --no-cpu --alt-steps 0 --steps 10 --warmup 1 > gpurun_out/scal/trace8.log 2>&1 || exit 2
python3 tools/trace_summary.py gpurun_out/scal/trace8/p8_kernel_trace.csv | head -8
