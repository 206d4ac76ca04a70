# Round 2: C5 with problems sharded over ranks (weak scaling, no data-path collective),
# rehearsed on ONE GPU with torchrun 2 ranks (--one-gpu: both on cuda:0); then N = 1.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2av
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 torchrun --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29631 \
  bench.py --gpus 2 --one-gpu --workload c5 --problems 512 --steps 2 --warmup 1 > $O/c5_n2.log 2>&1 || { tail -20 $O/c5_n2.log; exit 3; }
grep '"metric"' $O/c5_n2.log | cut -c1-900
timeout -k 10 300 python3 bench.py --workload c5 --problems 512 --steps 2 --warmup 1 --no-cpu --alt-steps 0 > $O/c5_n1.log 2>&1 || { tail -5 $O/c5_n1.log; exit 4; }
grep '"metric"' $O/c5_n1.log | cut -c1-400
