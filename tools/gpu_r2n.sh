# Round 2: Gram (C4 shard, panels) A/B of wave priority (libgmagg_prio1: producers at
# s_setprio 1; prio2: consumers), plus PMC passes for the effective clock
# (GRBM_GUI_ACTIVE / 8 / wall) and MFMA busy cycles, full kernel vs MFMA-only probe.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2n
L=$GRAFT_REPO_ROOT/byzantine_aircomp_amd
mkdir -p $O
step() {   # step <name> <timeout> <cmd...>: run, log, stop on anything but 0/1
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 $O/$name.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 10 --warmup 2 --no-cpu --no-check --alt-steps 0"
for v in base prio1 prio2 base2 prio1b; do
  case $v in base*) lib=$L/libgmagg.so;; prio1*) lib=$L/libgmagg_prio1.so;; prio2*) lib=$L/libgmagg_prio2.so;; esac
  GMAGG_LIB=$lib step ab_$v 200 python3 $B
  grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $O/ab_$v.log | tr '\n' ' '; echo
done
export GMAGG_GRAM_UNGUARDED=1
for dbg in 0 2; do
  export GMAGG_GRAM_DEBUG=$dbg
  step pmc_dbg$dbg 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $O/pmc_dbg$dbg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 3 --warmup 1 --no-cpu --no-check --alt-steps 0
  step kt_dbg$dbg 150 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_dbg$dbg -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c4-shard --algo gram --steps 3 --warmup 1 --no-cpu --no-check --alt-steps 0
done
