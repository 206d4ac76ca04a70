# Round 2, first GPU call: the new distributed / full-size tests, then the whole
# GPU suite, the 2-rank sharded run, the bench line and a one-GPU N=2 bench rehearsal.
# A test FAILURE (pytest exit 1) does not stop the script; any other non-zero
# status (timeout 124/137, abort 134, segfault 139) ends it at once.
set -o pipefail
O=gpurun_out/r2a
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -4 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step new 400 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_fullsize.py \
    tests/test_gpu_sharded.py -v --timeout 200 --timeout-method thread
step suite 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread \
    --deselect tests/test_gpu_fullsize.py
step two_rank 300 torchrun --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29611 tools/sharded_2rank.py
cat $O/two_rank.log | grep '"check"' || true
step bench 400 python -u bench.py
grep '"metric"' $O/bench.log || true
step bench_n2_rehearsal 400 torchrun --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29612 bench.py --gpus 2 --one-gpu --workload c3-small --steps 5 --warmup 2
grep '"metric"' $O/bench_n2_rehearsal.log || true
