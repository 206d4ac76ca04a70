# Round 2: where the Gram kernel's cycles go (C4 shard, panels, unguarded explicit Gram):
# SQ wait/active counters + GRBM_GUI_ACTIVE for the full kernel (DBG 0), producers
# only (DBG 1: no MFMAs) and consumers only (DBG 2: no loads).
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2o
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
cd /tmp && export TMPDIR=/tmp
export GMAGG_GRAM_UNGUARDED=1
for dbg in 0 1 2; do
  export GMAGG_GRAM_DEBUG=$dbg
  step pmc_dbg$dbg 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_dbg$dbg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 3 --warmup 1 --no-cpu --no-check --alt-steps 0
done
