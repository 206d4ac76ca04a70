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

hier() {
  # Round 5: the resident kernel's XCD-hierarchical gather (grids beyond one XCD) — parity,
  # then an interleaved A/B against the flat gather (GMAGG_RES_HIER=0) over shapes
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_resident_hier.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -3 $O/t.log
  for r in 1 2; do
    for h in 1 0; do
      GMAGG_RES_HIER=$h timeout -k 10 200 python -u tools/res_shape_bench.py \
        --shapes 50x7850,50x20000,50x48670,10x48670 --reps 5 >> $O/shapes.jsonl || return 3
    done
  done
  cat $O/shapes.jsonl
  # the batched kernel's groups (C5): sub-group gather (GMAGG_RB_HIER=1) against the flat one
  B="--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,1"
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=$B --variant hier= --variant flat=GMAGG_RB_HIER=0 \
    --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 4; }
  tail -3 $O/ab_c5.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=$B,--reading,aircomp --variant hier= \
    --variant flat=GMAGG_RB_HIER=0 --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 5; }
  tail -3 $O/ab_c5air.log
}

hier2() {
  # Round 5: where the single-problem hierarchical gather starts to pay (grid size x values
  # per block), and the C5 AirComp launch's HBM traffic with / without the batched one
  for r in 1 2; do
    for h in 1 0; do
      GMAGG_RES_HIER=$h timeout -k 10 200 python -u tools/res_shape_bench.py \
        --shapes 50x30000,50x40000,50x60000,30x48670,40x48670,20x48670 --reps 5 >> $O/shapes.jsonl || return 3
    done
  done
  cat $O/shapes.jsonl
  for h in 1 0; do
    for c in FETCH_SIZE WRITE_SIZE; do
      GMAGG_RB_HIER=$h timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_h${h}_$c -o p -- \
        python3 bench.py --workload c5 --reading aircomp --steps 1 --warmup 0 $B_FAST --no-check \
        > $O/pmc_h${h}_$c.log 2>&1 || return 4
    done
    python3 tools/pmc_summary.py $(find $O/pmc_h${h}_FETCH_SIZE -name "*counter_collection.csv" | head -1) \
      $(find $O/pmc_h${h}_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/pmc_c5air_h$h.json \
      "c5air hier=$h" || return 5
  done
}

split() {
  # Round 5: the batched kernel's split-scope exchange (GMAGG_RB_HIER=2: one hop, each
  # granule agent-scope + L2-kept, read from its XCD's copy) against the flat one: parity,
  # C5 A/B (both readings), the AirComp launch's HBM traffic
  timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_resident_hier.py -k batched > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  B="--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,1"
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=$B,--reading,aircomp --variant split=GMAGG_RB_HIER=2 \
    --variant flat= --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 5; }
  tail -2 $O/ab_c5air.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=$B --variant split=GMAGG_RB_HIER=2 --variant flat= \
    --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 4; }
  tail -2 $O/ab_c5.log
  for c in FETCH_SIZE WRITE_SIZE; do
    GMAGG_RB_HIER=2 timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_h2_$c -o p -- \
      python3 bench.py --workload c5 --reading aircomp --steps 1 --warmup 0 $B_FAST --no-check \
      > $O/pmc_h2_$c.log 2>&1 || return 6
  done
  python3 tools/pmc_summary.py $(find $O/pmc_h2_FETCH_SIZE -name "*counter_collection.csv" | head -1) \
    $(find $O/pmc_h2_WRITE_SIZE -name "*counter_collection.csv" | head -1) $O/pmc_c5air_h2.json \
    "c5air split" | grep resident_batched
  # the single-problem kernel's split scope (GMAGG_RES_SPLIT=1) on the grids below the
  # hierarchical gather's range
  for r in 1 2; do
    for sp in 1 0; do
      GMAGG_RES_SPLIT=$sp timeout -k 10 200 python -u tools/res_shape_bench.py \
        --shapes 50x20000,50x30000,30x48670,10x48670 --reps 5 | sed "s/}$/, \"split\": $sp}/" >> $O/shapes.jsonl || return 7
    done
  done
  cat $O/shapes.jsonl
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

hier_floor() {
  # Round 5: the exchange floors of the resident kernel's gathers beyond one XCD (libgmagg_floor.so:
  # make alt ALT_ONLY=resident ALT_FLAGS=-DGMK_RES_DBG=7) and a longer level-2 poll back-off
  # (libgmagg_sl4.so: ALT_FLAGS=-DGMK_RES_L2SLEEP=4)
  for r in 1 2; do
    for lib in product floor sl4; do
      L=""; [ $lib != product ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$lib.so"
      for ex in "hier:GMAGG_RES_HIER=2" "split:GMAGG_RES_HIER=0" "flat:GMAGG_RES_HIER=0 GMAGG_RES_SPLIT=0"; do
        n=${ex%%:*}; e=${ex#*:}
        env $L $e timeout -k 10 200 python -u tools/res_shape_bench.py --shapes 50x48670,50x20000 --reps 5 \
          | sed "s/}$/, \"lib\": \"$lib\", \"ex\": \"$n\"}/" >> $O/floor.jsonl || return 3
      done
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/floor.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["lib"], r["ex"])].append(r["us_per_iteration"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.2f}" for v in acc[k]))
PY
}

poll_ab() {
  # Round 5: poll pressure of the resident kernel's multi-XCD gathers — variant libraries
  # (make alt ALT_ONLY=resident ALT_FLAGS=...): libgmagg_sl4all.so -DGMK_RES_SLEEP=4,
  # libgmagg_sl10all.so -DGMK_RES_SLEEP=10, libgmagg_poll1.so -DGMK_RES_POLL1=1
  for r in 1 2; do
    for lib in product sl4all sl10all poll1; do
      L=""; [ $lib != product ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$lib.so"
      for ex in "auto:GMAGG_RES_HIER=1" "hier:GMAGG_RES_HIER=2" "flat:GMAGG_RES_HIER=0 GMAGG_RES_SPLIT=0"; do
        n=${ex%%:*}; e=${ex#*:}
        env $L $e timeout -k 10 200 python -u tools/res_shape_bench.py --shapes 50x7850,50x48670,50x20000 --reps 5 \
          | sed "s/}$/, \"lib\": \"$lib\", \"ex\": \"$n\"}/" >> $O/poll.jsonl || return 3
      done
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/poll.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["ex"], r["lib"])].append(r["us_per_iteration"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.2f}" for v in acc[k]))
PY
}

c2_ab() {
  # C2's resident kernel, this build against libgmagg_r4res.so (the round-4 resident.hip linked
  # with the same other objects): interleaved bench A/B, three rounds
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 \
    --variant now= --variant r4=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_r4res.so --out $O/ab_c2.jsonl \
    > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 1; }
  tail -2 $O/ab_c2.log
}

f3_ab() {
  # f3 selection: this build against libgmagg_old.so (the previous build, copied aside):
  # the f3 GPU tests, then select_bench interleaved, three rounds
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_other_aggregators.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for r in 1 2 3; do
    for lib in new old; do
      L=""; [ $lib = old ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_old.so"
      env $L timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 5 \
        | sed "s/}$/, \"lib\": \"$lib\"}/" >> $O/sel.jsonl || return 2
    done
  done
  cat $O/sel.jsonl
}

tm_variants() {
  # the trimmed mean's selection after the round-5 tail change: the one-column kernel against
  # the column-pair one (GMAGG_SELECT_1COL=0), and the histogram schedule (libgmagg_h1.so:
  # make alt ALT_ONLY=coordinate ALT_FLAGS=-DGMK_SELECT_HIST=1, libgmagg_h0.so: =0), and the
  # counting steps' ballot share (libgmagg_nbN.so: ALT_FLAGS=-DGMK_SELECT_NBALLOT=N)
  for r in 1 2; do
    for v in "def:" "pair:GMAGG_SELECT_1COL=0" "h1:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_h1.so" \
             "h0:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_h0.so" \
             "h1pair:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_h1.so GMAGG_SELECT_1COL=0" \
             "nb4:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_nb4.so" "nb8:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_nb8.so"; do
      n=${v%%:*}; e=${v#*:}
      env $e timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 5 \
        | sed "s/}$/, \"v\": \"$n\"}/" >> $O/sel.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/sel.jsonl"):
    r = json.loads(l)
    acc[(r["agg"], r["K"], r["v"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

krum() {
  # Round 5: Krum through the Gram MFMA kernel against the exact pair-distance path over
  # (K, d), then the kernel trace of both paths at K = 256 x 4M
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_krum_gram.py \
    > $O/t.log 2>&1 || { tail -30 $O/t.log; return 3; }
  tail -1 $O/t.log
  timeout -k 10 600 python -u tools/krum_bench.py --reps 5 > $O/krum.jsonl 2> $O/krum.err || { tail -20 $O/krum.err; return 1; }
  cat $O/krum.jsonl
  GMAGG_KRUM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o t -- \
    python3 tools/krum_bench.py --shapes 256x4194304 --reps 5 > $O/trace.log 2>&1 || return 2
  cut -c1-150 $O/trace/t_kernel_stats.csv | head -14
}

st_ab() {
  # Round 5: the staged-transpose selection kernel (GMAGG_SELECT_ST=1: the median, default;
  # 2: both modes; 0: the round-4 tiles): the f3 tests under each, then select_bench
  # interleaved over K
  for v in 0 2; do
    GMAGG_SELECT_ST=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
      tests/test_gpu_other_aggregators.py > $O/t$v.log 2>&1 || { tail -30 $O/t$v.log; return 1; }
    tail -1 $O/t$v.log
  done
  for r in 1 2 3; do
    for v in 0 1; do
      GMAGG_SELECT_ST=$v timeout -k 10 200 python -u tools/select_bench.py --K 2000 1000 400 256 200 --reps 5 \
        | sed "s/}$/, \"st\": $v}/" >> $O/sel.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/sel.jsonl"):
    r = json.loads(l)
    acc[(r["agg"], r["K"], r["st"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

st_wpe() {
  # the staged-transpose median (GMAGG_SELECT_ST=2) at the compiler's occupancy (6 waves per
  # SIMD) against forced 7 / 8 (libgmagg_wpeN.so: make alt ALT_ONLY=coordinate
  # ALT_FLAGS=-DGMK_SELECT_ST_WPE=N)
  for r in 1 2 3; do
    for v in "st0:GMAGG_SELECT_ST=0" "st2:GMAGG_SELECT_ST=2" \
             "wpe7:GMAGG_SELECT_ST=2 GMAGG_LIB=byzantine_aircomp_amd/libgmagg_wpe7.so" \
             "wpe8:GMAGG_SELECT_ST=2 GMAGG_LIB=byzantine_aircomp_amd/libgmagg_wpe8.so"; do
      n=${v%%:*}; e=${v#*:}
      env $e timeout -k 10 120 python -u tools/select_bench.py --K 1000 --reps 5 \
        | sed "s/}$/, \"v\": \"$n\"}/" >> $O/sel.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/sel.jsonl"):
    r = json.loads(l)
    acc[(r["agg"], r["K"], r["v"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

st_pf() {
  # the staged median with the next round's loads in flight (libgmagg_alt.so: make alt
  # ALT_ONLY=coordinate ALT_FLAGS=-DGMK_SELECT_ST_PREFETCH=1) against the default
  for r in 1 2 3; do
    for v in "def:" "pf:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so"; do
      n=${v%%:*}; e=${v#*:}
      env $e timeout -k 10 120 python -u tools/select_bench.py --K 1000 400 256 --reps 5 \
        | sed "s/}$/, \"v\": \"$n\"}/" >> $O/sel.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/sel.jsonl"):
    r = json.loads(l)
    if r["agg"] == "median":
        acc[(r["agg"], r["K"], r["v"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

sel_keys() {
  # this build's selection kernels against the previous build (libgmagg_old.so, copied
  # aside); the f3 tests first
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_other_aggregators.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for r in 1 2 3; do
    for v in "new:" "old:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_old.so"; do
      n=${v%%:*}; e=${v#*:}
      env $e timeout -k 10 200 python -u tools/select_bench.py --K 1000 400 256 --reps 5 \
        | sed "s/}$/, \"v\": \"$n\"}/" >> $O/sel.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/sel.jsonl"):
    r = json.loads(l)
    acc[(r["agg"], r["K"], r["v"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

st_tm() {
  # the trimmed mean on the staged kernel (GMAGG_SELECT_ST=2) against the default
  for r in 1 2 3; do
    for v in 1 2; do
      GMAGG_SELECT_ST=$v timeout -k 10 200 python -u tools/select_bench.py --K 1000 400 256 --reps 5 \
        | sed "s/}$/, \"st\": $v}/" >> $O/sel.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/sel.jsonl"):
    r = json.loads(l)
    acc[(r["agg"], r["K"], r["st"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

cpb_ab() {
  # Round 5: the resident kernel beyond one XCD at smaller blocks (GMAGG_RES_CPB = chunks of
  # 128 columns per block: 4 is AUTO's choice at d = 48,670 -> 96 blocks; 2 -> 191, 1 -> 381)
  # under each gather
  for r in 1 2; do
    for cpb in 4 2 1; do
      for ex in "auto:GMAGG_RES_HIER=1" "split:GMAGG_RES_HIER=0" "flat:GMAGG_RES_HIER=0 GMAGG_RES_SPLIT=0"; do
        n=${ex%%:*}; e=${ex#*:}
        env GMAGG_RES_CPB=$cpb $e timeout -k 10 200 python -u tools/res_shape_bench.py --shapes 50x48670,50x30000 --reps 5 \
          | sed "s/}$/, \"cpb\": $cpb, \"ex\": \"$n\"}/" >> $O/cpb.jsonl || return 3
      done
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/cpb.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["cpb"], r["ex"], r["exchange"], r["algo"])].append(r["us_per_iteration"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.2f}" for v in acc[k]))
PY
}

cpb_ab2() {
  # the resident kernel's block size beyond one XCD under AUTO's exchange: 4 chunks per
  # block (AUTO's current choice, the fewest blocks) against 2, over shapes
  for r in 1 2; do
    for cpb in 4 2; do
      GMAGG_RES_CPB=$cpb timeout -k 10 300 python -u tools/res_shape_bench.py \
        --shapes 50x20000,50x40000,50x48670,50x60000,40x48670,64x48670,64x30000 --reps 5 \
        | sed "s/}$/, \"cpb\": $cpb}/" >> $O/cpb.jsonl || return 3
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/cpb.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["cpb"], r["exchange"], r["algo"])].append(r["us_per_iteration"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.2f}" for v in acc[k]))
PY
}

cpb_ab3() {
  # odd d (the 1-value tile, V = 1): 8 chunks per block (AUTO's largest valid) against 4 and 2
  for r in 1 2; do
    for cpb in 8 4 2; do
      GMAGG_RES_CPB=$cpb timeout -k 10 300 python -u tools/res_shape_bench.py \
        --shapes 50x48671,50x30001,50x20001 --reps 5 | sed "s/}$/, \"cpb\": $cpb}/" >> $O/cpb.jsonl || return 3
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/cpb.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["cpb"], r["exchange"], r["algo"])].append(r["us_per_iteration"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.2f}" for v in acc[k]))
PY
}

halve_ab() {
  # the resident block rule (half the columns per block in the hierarchical gather's range)
  # against the largest tile (GMAGG_RES_HALVE=0), over shapes incl. K <= 32 tiles
  for r in 1 2; do
    for h in 1 0; do
      GMAGG_RES_HALVE=$h timeout -k 10 300 python -u tools/res_shape_bench.py \
        --shapes 10x48670,20x48670,30x48670,32x60000,50x48670,64x60000,50x65000 --reps 5 \
        | sed "s/}$/, \"halve\": $h}/" >> $O/h.jsonl || return 3
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/h.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["halve"], r["exchange"], r["algo"])].append(r["us_per_iteration"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.2f}" for v in acc[k]))
PY
}

krum_ab() {
  # the Gram Krum path of this build against the previous build (libgmagg_old.so, copied
  # aside): its tests, then krum_bench interleaved
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_krum_gram.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for r in 1 2 3; do
    for v in "new:" "old:GMAGG_LIB=byzantine_aircomp_amd/libgmagg_old.so"; do
      n=${v%%:*}; e=${v#*:}
      env $e timeout -k 10 300 python -u tools/krum_bench.py --shapes 256x4194304,256x1048576,64x1048576 \
        --reps 5 | grep '"gram"' | sed "s/}$/, \"v\": \"$n\"}/" >> $O/k.jsonl || return 2
    done
  done
  python3 - "$O" <<'PY'
import collections, json, sys
acc = collections.defaultdict(list)
for l in open(sys.argv[1] + "/k.jsonl"):
    r = json.loads(l)
    acc[(r["K"], r["d"], r["v"])].append(r["ms"])
for k in sorted(acc):
    print(k, " ".join(f"{v:.3f}" for v in acc[k]))
PY
}

[ $# -ge 1 ] && declare -F "$1" > /dev/null || { echo "usage: $0 SET [TAG]  (sets: $(declare -F | awk '{print $3}' | tr '\n' ' '))"; exit 2; }
O=gpurun_out/${2:-$1}
mkdir -p "$O"
"$1"
