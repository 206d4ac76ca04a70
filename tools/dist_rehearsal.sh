# One-GPU rehearsal of bench.py's multi-rank path (process group, RCCL comm, d-shard,
# per-iteration ncclAllReduce, max-over-ranks timing, teardown).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --dist --no-cpu --steps 5 --warmup 1 > gpurun_out/dist_plain.json 2> gpurun_out/dist_plain.err || { echo "plain rc=$?"; tail -20 gpurun_out/dist_plain.err; exit 1; }
echo "plain rc=0"; cat gpurun_out/dist_plain.json
timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29544 bench.py --gpus 1 --dist --no-cpu --steps 5 --warmup 1 > gpurun_out/dist_torchrun.json 2> gpurun_out/dist_torchrun.err || { echo "torchrun rc=$?"; tail -20 gpurun_out/dist_torchrun.err; exit 1; }
echo "torchrun rc=0"; cat gpurun_out/dist_torchrun.json
timeout -k 10 300 python -u bench.py --dist --workload c4-shard --no-cpu --steps 5 --warmup 1 > gpurun_out/dist_c4.json 2> gpurun_out/dist_c4.err || { echo "c4 rc=$?"; tail -20 gpurun_out/dist_c4.err; exit 1; }
echo "c4 rc=0"; cat gpurun_out/dist_c4.json
