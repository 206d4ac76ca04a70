# Round 2 (late): the N > 1 bench path with the final code (panel staging in api.hip), rehearsed
# on one GPU: 2 and 4 ranks (gloo + the torch.distributed transport), C3 recipe at a
# reduced width; then the 2-rank sharded check against the single-process call.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2as
mkdir -p $O
cd $GRAFT_REPO_ROOT
for n in 2 4; do
  timeout -k 10 400 torchrun --nnodes 1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2961$n \
    bench.py --gpus $n --one-gpu --workload c3-small --steps 5 --warmup 2 --soak 3 > $O/bench_n$n.log 2>&1 || { tail -20 $O/bench_n$n.log; exit 3; }
  grep '"metric"' $O/bench_n$n.log | cut -c1-400
done
timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29619 tools/sharded_2rank.py > $O/two_rank.log 2>&1 || { tail -20 $O/two_rank.log; exit 4; }
grep '"check"' $O/two_rank.log | cut -c1-300
