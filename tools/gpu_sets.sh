#!/bin/bash
# The GPU-box measurement sets behind the CURRENT numbers in DESIGN.md (§3-§4).  Older
# one-off A/B sets are in git history (this file before round 5); their results are in
# DESIGN.md §9 and profiles/.
#
#   bash tools/gpu_sets.sh SET [TAG]     e.g.  bash tools/gpu_sets.sh closing r5s2z
#
# Output goes to gpurun_out/TAG (default: the set's name).  Every GPU step runs under its
# own time limit and a set stops at its first failing step.  Probe sets that name
# libgmagg_alt.so need the matching `make alt ALT_FLAGS=...` build first (in the comment).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 9
export TMPDIR=/tmp
B_FAST="--no-cpu --alt-steps 0 --soak 0"

closing() {
  # GPU suite + smoke + the default bench line (tools/final_check.sh), every BASELINE
  # workload's line, C2's kernel trace and the f3 timings (DESIGN.md §4's table)
  bash tools/final_check.sh || return $?
  for w in "c2:--workload c2" "c5:--workload c5" "c5air:--workload c5 --reading aircomp" \
           "c4:--workload c4 --steps 5 --warmup 1" "c4shard:--workload c4-shard"; do
    n=${w%%:*}; a=${w#*:}
    timeout -k 10 600 python -u bench.py $a > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; return 2; }
    cut -c1-300 $O/bench_$n.json
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o t -- \
    python3 bench.py --workload c2 $B_FAST > $O/trace_c2.log 2>&1 || return 3
  head -3 $O/trace_c2/t_kernel_stats.csv
  timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 3 > $O/select.jsonl 2> $O/select.err || return 4
  cat $O/select.jsonl
}

traces() {
  # rocprofv3 --kernel-trace --stats of the C3 (default), C5 and C4 bench lines: each line's
  # HIP-event launch time paired with rocprof's average for the same kernel
  for w in "c3:" "c5:--workload c5" "c4:--workload c4 --steps 3 --warmup 1"; do
    n=${w%%:*}; a=${w#*:}
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o t -- \
      python3 bench.py $a $B_FAST > $O/trace_$n.json 2> $O/trace_$n.err || return 1
    head -4 $O/trace_$n/t_kernel_stats.csv | cut -c1-200
    python3 -c "import json;l=json.load(open('$O/trace_$n.json'));print('$n bench avg_launch_us', l['roofline'].get('avg_launch_us'))"
  done
}

pmc() {
  # HBM traffic of the dominant kernels (one counter per pass; tools/pmc_summary.py applies
  # the gfx950 FETCH_SIZE correction): C3 panels, C4 whole job, C5 both readings
  for w in "c3:" "c4:--workload c4 --steps 2 --warmup 1" "c5:--workload c5 --steps 1 --warmup 0" \
           "c5air:--workload c5 --reading aircomp --steps 1 --warmup 0" "c2:--workload c2 --steps 3 --warmup 1"; do
    n=${w%%:*}; a=${w#*:}
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${n}_$c -o p -- \
        python3 bench.py $a $B_FAST --no-check > $O/pmc_${n}_$c.log 2>&1 || return 1
    done
  done
  ls $O
}

floors() {
  # Latency floors of the resident kernels: the exchange alone (compute phases skipped).
  # Build first: make alt ALT_ONLY="resident resident_batched" ALT_FLAGS="-DGMK_RES_DBG=7 -DGMK_RB_DBG_VARIANTS"
  for v in product alt; do
    L=""; [ $v = alt ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so"
    env $L GMAGG_RB_DBG=7 timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B_FAST --no-check \
      > $O/c2_$v.json 2> $O/c2_$v.err || return 2
    env $L GMAGG_RB_DBG=7 timeout -k 10 300 python -u tools/rb_probe.py > $O/rb_$v.log 2>&1 || return 3
  done
  tail -3 $O/rb_*.log
}

select_pmc() {
  # Where the f3 selection's time goes (issue- or latency-bound?)
  timeout -k 10 120 python -u tools/select_bench.py --K 1000 --reps 3 > $O/select.log 2>&1 || return 5
  cat $O/select.log
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY \
    --output-format csv -d $O/pmc_sel -o p -- python3 tools/select_bench.py --K 1000 --reps 1 > $O/pmc_sel.log 2>&1 || return 6
}

loop() {
  # the training loop (rows f2/f4) and its kernel trace
  timeout -k 10 300 python -u tools/loop_bench.py --steps 20 > $O/loop.jsonl 2> $O/loop.err || { tail -20 $O/loop.err; return 2; }
  cut -c1-60,150-260 $O/loop.jsonl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loop -o t -- \
    python3 tools/loop_bench.py --steps 20 > $O/trace_loop.log 2>&1 || return 3
  head -4 $O/trace_loop/t_kernel_stats.csv
}

c4_pmc() {
  # Round 5: the whole-C4 Gram partial's clock and MFMA occupancy —
  # effective clock = GRBM_GUI_ACTIVE / 8 / kernel time, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES
  # / (cycles x SIMDs); a kernel trace of the same command for the time
  A="--workload c4 --steps 2 --warmup 1 $B_FAST --no-check"
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- python3 bench.py $A \
    > $O/trace.json 2> $O/trace.err || { tail -5 $O/trace.err; return 1; }
  grep -i "gram" $O/trace/t_kernel_stats.csv | cut -c1-200
  timeout -s KILL 600 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    SQ_INSTS_VALU SQ_INSTS_MFMA --output-format csv -d $O/pmc -o p -- python3 bench.py $A > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; return 2; }
  python3 - "$O" <<'PY'
import collections, csv, glob, sys
o = sys.argv[1]
f = glob.glob(o + "/pmc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    if "gram" in r["Kernel_Name"]:
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in acc.items():
    print(k, {c: sum(x) / len(x) for c, x in v.items()})
PY
}

[ $# -ge 1 ] && declare -F "$1" > /dev/null || { echo "usage: $0 SET [TAG]  (sets: $(declare -F | awk '{print $3}' | tr '\n' ' '))"; exit 2; }
O=gpurun_out/${2:-$1}
mkdir -p "$O"
"$1"
