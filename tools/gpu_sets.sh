#!/bin/bash
# The GPU-box measurement sets behind profiles/ (one function per set, named by the
# profile prefix it produced; round 3 kept one script per set under tools/runs/).
#
#   bash tools/gpu_sets.sh SET        e.g.  bash tools/gpu_sets.sh r4s1f
#
# Every set writes under gpurun_out/, runs each GPU step under its own time limit and
# stops at the first failing step.  Probe sets that name libgmagg_alt.so need the
# matching `make alt ALT_FLAGS=...` build first (the flags are in the set's comment).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}" || exit 9
export TMPDIR=/tmp

r3s2b() {
  o=gpurun_out/r3s2b; mkdir -p $o
  timeout -k 10 400 python tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant coop= --variant plain=GMAGG_RES_COOP=0 --out $o/ab_c2_coop.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -2 $o/ab.log
  GMAGG_RES_COOP=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/c2plain -o t -- python3 bench.py --workload c2 --no-cpu --soak 0 --alt-steps 0 > $o/c2plain.log 2>&1; echo "c2 plain-launch trace return $?"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/probe_plain -o t -- ./tools/coop_exit_probe plain > $o/probe_plain.log 2>&1; echo "probe plain return $?"
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $o/probe_coop -o t -- ./tools/coop_exit_probe coop > $o/probe_coop.log 2>&1; echo "probe coop return $?"
}

r3s2c() {
  o=gpurun_out/r3s2c; mkdir -p $o
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py > $o/t_resident.log 2>&1; rc=$?
  tail -5 $o/t_resident.log; grep -E "FAILED|Error|assert" $o/t_resident.log | head -20
  [ $rc -ne 0 ] && return $rc
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_batched.py tests/test_gpu_c5_fullsize.py > $o/t_batched.log 2>&1 || { tail -30 $o/t_batched.log; return 1; }
  tail -2 $o/t_batched.log
  timeout -k 10 600 python -u bench.py --workload c5 --no-cpu --alt-steps 0 --soak 0 > $o/c5_res.json 2> $o/c5_res.err || { tail -20 $o/c5_res.err; return 1; }
  python -c "import json;l=json.load(open('$o/c5_res.json'));print('resident c5', l['value'], l['ms_per_step'], l['check'], l['config']['groups'])"
  GMAGG_BATCH_RESIDENT=0 timeout -k 10 600 python -u bench.py --workload c5 --no-cpu --alt-steps 0 --soak 0 > $o/c5_stream.json 2> $o/c5_stream.err || { tail -20 $o/c5_stream.err; return 1; }
  python -c "import json;l=json.load(open('$o/c5_stream.json'));print('stream c5', l['value'], l['ms_per_step'])"
}

r3s2f() {
  o=gpurun_out/r3s2f; mkdir -p $o
  for dbg in 0 1 2 4 8 16 31; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $o/dbg$dbg.log 2>&1 || { tail -5 $o/dbg$dbg.log; return 1; }
    grep fit $o/dbg$dbg.log
  done
}

r3s2g() {
  o=gpurun_out/r3s2g; mkdir -p $o
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py > $o/t_resident.log 2>&1 || { tail -30 $o/t_resident.log; return 1; }
  tail -1 $o/t_resident.log
  for dbg in 0 1 4; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $o/dbg$dbg.log 2>&1 || { tail -5 $o/dbg$dbg.log; return 1; }
    grep fit $o/dbg$dbg.log
  done
  timeout -k 10 600 python -u bench.py --workload c5 --no-cpu --alt-steps 0 --soak 0 > $o/c5.json 2> $o/c5.err || { tail -20 $o/c5.err; return 1; }
  python -c "import json;l=json.load(open('$o/c5.json'));print('c5', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline']['aggregation_frac'], l['check']['ok'], l['config']['groups'])"
}

r3s2h() {
  o=gpurun_out/r3s2h; mkdir -p $o
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant oma2= --variant oma1=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -3 $o/ab.log
}

r3s2i() {
  o=gpurun_out/r3s2i; mkdir -p $o
  timeout -k 10 300 python -u tools/rb_probe.py > $o/cur.log 2>&1 || { tail -5 $o/cur.log; return 1; }
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 300 python -u tools/rb_probe.py > $o/old.log 2>&1 || { tail -5 $o/old.log; return 1; }
  echo cur; grep fit $o/cur.log; echo old; grep fit $o/old.log
}

r3s2j() {
  o=gpurun_out/r3s2j; mkdir -p $o
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_c5_fullsize.py > $o/t.log 2>&1 || { tail -30 $o/t.log; return 1; }
  tail -1 $o/t.log
  timeout -k 10 300 python -u tools/rb_probe.py --quick > $o/probe_cur.log 2>&1 || { tail -5 $o/probe_cur.log; return 1; }
  grep fit $o/probe_cur.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant cur= --variant old=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -2 $o/ab.log
}

r3s2l() {
  o=gpurun_out/r3s2l; mkdir -p $o
  timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_batched.py tests/test_gpu_c5_fullsize.py > $o/t.log 2>&1; rc=$?
  tail -3 $o/t.log; grep -E "^FAILED|Error" $o/t.log | head
  [ $rc -ne 0 ] && return $rc
  timeout -k 10 900 python -u bench.py --workload c5 --no-cpu --soak 0 > $o/c5.json 2> $o/c5.err || { tail -20 $o/c5.err; return 1; }
  python -c "import json;l=json.load(open('$o/c5.json'));print('c5', l['value'], json.dumps(l['alt_layout']))"
}

r3s2n() {
  o=gpurun_out/r3s2n; mkdir -p $o
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant perwave= --variant wave0=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -2 $o/ab.log
}

r3s2o() {
  o=gpurun_out/r3s2o; mkdir -p $o
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_training.py tests/test_gpu_resident_batched.py > $o/t.log 2>&1 || { tail -30 $o/t.log; return 1; }
  tail -1 $o/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant fast= --variant prev=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c2.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -2 $o/ab.log
}

r3s2p() {
  o=gpurun_out/r3s2p; mkdir -p $o
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py > $o/t.log 2>&1 || { tail -30 $o/t.log; return 1; }
  tail -1 $o/t.log
  for dbg in 0 128 256 32; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $o/dbg$dbg.log 2>&1 || { tail -5 $o/dbg$dbg.log; return 1; }
    grep fit $o/dbg$dbg.log
  done
  timeout -k 10 200 python -u tools/rb_probe.py --quick > $o/cur.log 2>&1 || { tail -5 $o/cur.log; return 1; }
  grep fit $o/cur.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant cur= --variant prev=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -2 $o/ab.log
}

r3s2q() {
  o=gpurun_out/r3s2q; mkdir -p $o
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant pf0= --variant pf10=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --variant pf5=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt2.so --out $o/ab_c5.jsonl > $o/ab.log 2>&1 || { tail -20 $o/ab.log; return 1; }
  tail -3 $o/ab.log
  timeout -k 10 300 python -u tools/loop_bench.py > $o/loop.log 2>&1 || { tail -20 $o/loop.log; return 1; }
  tail -8 $o/loop.log
}

r3s3_c2_layouts() {
  # C2 (AirComp gm, K=50, d=7850, 1000 iterations): rows (C2 single resident kernel) vs panels
  # (the batched resident kernel at P = 1), interleaved twice on one box
  mkdir -p gpurun_out
  for i in 1 2; do
    timeout -k 10 120 python -u bench.py --workload c2 --steps 100 --warmup 5 --alt-steps 0 \
      >> gpurun_out/r3s3_c2_rows.jsonl 2>> gpurun_out/r3s3_c2.err || return $?
    timeout -k 10 120 python -u bench.py --workload c2 --layout panels --steps 100 --warmup 5 \
      --alt-steps 0 >> gpurun_out/r3s3_c2_panels.jsonl 2>> gpurun_out/r3s3_c2.err || return $?
  done
}

r3s3_c5air_pmc() {
  # HBM traffic of the C5 AirComp reading's resident gm kernel: FETCH_SIZE and WRITE_SIZE,
  # each in its own pass, then tools/pmc_summary.py
  O=gpurun_out/c5air_pmc
  mkdir -p $O
  B="bench.py --workload c5 --reading aircomp --steps 1 --warmup 0 --no-cpu --alt-steps 0 --no-check"
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o p -- python3 $B > $O/f.json 2> $O/f.err &&
  timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o p -- python3 $B > $O/w.json 2> $O/w.err &&
  python3 tools/pmc_summary.py $O/f/p_counter_collection.csv $O/w/p_counter_collection.csv $O/pmc.json "c5 aircomp reading, panels, resident" > $O/summary.txt 2>&1
}

r3s3_c5air_trace() {
  # kernel trace of the C5 AirComp reading (gm, 1000 iterations per noisy problem) on the
  # spill-free batched resident tile
  mkdir -p gpurun_out/c5air
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5air/prof -o run -- \
    python3 bench.py --workload c5 --reading aircomp --steps 1 --warmup 1 --no-cpu --alt-steps 0 \
    > gpurun_out/c5air/bench.json 2> gpurun_out/c5air/bench.err
}

r3s3_panels1() {
  # single-call panels -> batched resident kernel (P = 1): the panel / pre-noise tests, then the
  # training loop bench on both layouts
  mkdir -p gpurun_out
  timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_panels.py tests/test_gpu_resident_batched.py \
    "tests/test_gpu_weiszfeld.py::test_pre_oma_equals_oma_then_gm2" > gpurun_out/r3s3_panels1.log 2>&1 &&
  timeout -k 10 200 python -u tools/loop_bench.py > gpurun_out/r3s3_loop.jsonl 2>&1
}

r3s3_rb_draws() {
  # resident batched, AirComp draws drawn after the publish + r_k in LDS (no scratch at KR=50
  # MODE 1) vs the previous library (libgmagg_alt.so: 352 B/lane of scratch): C2 on panels
  # (P = 1), then C5 (gm2, must not move), C5's AirComp reading (gm, 1000 iterations); then the resident-batched GPU tests
  mkdir -p gpurun_out
  L=$PWD/byzantine_aircomp_amd/libgmagg_alt.so
  timeout -k 10 300 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--layout,panels,--steps,100,--warmup,5,--alt-steps,0,--no-cpu \
    --variant new= --variant old=GMAGG_LIB=$L --out gpurun_out/r3s3_rb_draws_c2_ab.jsonl > gpurun_out/r3s3_rb_draws_c2_ab.txt 2>&1 &&
  timeout -k 10 300 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--no-cpu,--alt-steps,0 \
    --variant new= --variant old=GMAGG_LIB=$L --out gpurun_out/r3s3_rb_draws_c5_ab.jsonl > gpurun_out/r3s3_rb_draws_c5_ab.txt 2>&1 &&
  timeout -k 10 400 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--steps,1,--warmup,1,--no-cpu,--alt-steps,0 \
    --variant new= --variant old=GMAGG_LIB=$L --out gpurun_out/r3s3_rb_draws_c5air_ab.jsonl > gpurun_out/r3s3_rb_draws_c5air_ab.txt 2>&1 &&
  timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
    tests/test_gpu_resident_batched.py tests/test_gpu_panels.py > gpurun_out/r3s3_rb_draws_tests.log 2>&1
}

r4s1e() {
  O=gpurun_out/r4s1e; mkdir -p $O; export TMPDIR=/tmp
  timeout -k 10 300 python -u -m pytest tests/test_gpu_weiszfeld.py -q -x --timeout 200 --timeout-method thread -rf -p no:cacheprovider -k "c4_recipe or guard or gram_split" > $O/pytest.log 2>&1; tail -3 $O/pytest.log
  GMAGG_GUARD_DEBUG=1 timeout -k 10 400 python -u bench.py --workload c4 --steps 5 --warmup 1 --no-cpu > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; return 3; }
  grep "gram guard" $O/c4.err | tail -2; cut -c1-600 $O/c4.json
  for dbg in 0 7; do GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $O/rb_probe_dbg$dbg.log 2>&1 || return 4; tail -1 $O/rb_probe_dbg$dbg.log; done
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/c2_exchange_only.json 2> $O/c2x.err || return 5
  timeout -k 10 200 python -u bench.py --workload c2 --steps 10 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/c2.json 2> $O/c2.err || return 6
  python -c "
  import json
  for f in ('c2_exchange_only','c2'):
      d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['roofline'].get('us_per_iteration'))"
}

r4s1f() {
  # Round 4 session 1: latency-roofline probes (exchange floor, VALU instruction counts)
  # and the whole-C4 Gram job's trace + PMC traffic.
  O=gpurun_out/r4s1f; mkdir -p $O; export TMPDIR=/tmp
  B="--no-cpu --no-check --alt-steps 0 --soak 0"
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_exchange_only.json 2> $O/c2x.err || return 2
  timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_tolneg.json 2> $O/c2.err || return 3
  for w in "c2:--workload c2 --steps 3" "c5air:--workload c5 --reading aircomp --steps 1 --warmup 0" "c5pre:--workload c5 --steps 1 --warmup 0"; do
    n=${w%%:*}; a=${w#*:}
    timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc_valu_$n -o p -- python3 bench.py $a $B > $O/pmc_valu_$n.log 2>&1 || return 4
  done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o t -- python3 bench.py --workload c4 --steps 3 --warmup 1 $B > $O/trace_c4.log 2>&1 || return 5
  head -5 $O/trace_c4/t_kernel_stats.csv
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_c4_$c -o p -- python3 bench.py --workload c4 --steps 2 --warmup 1 $B > $O/pmc_c4_$c.log 2>&1 || return 6
  done
  ls -R $O | head -40
}

r4s1g() {
  # Round 4 session 1: the closing check (GPU suite, smoke, default bench), then PMC of
  # the f3 selection kernels (issue- or latency-bound?).
  bash tools/final_check.sh || return $?
  O=gpurun_out/r4s1g; mkdir -p $O; export TMPDIR=/tmp
  timeout -k 10 120 python -u tools/select_bench.py --K 1000 --reps 3 > $O/select.log 2>&1 || return 5
  cat $O/select.log
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/pmc_sel -o p -- python3 tools/select_bench.py --K 1000 --reps 1 > $O/pmc_sel.log 2>&1 || return 6
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_ACTIVE_INST_ANY --output-format csv -d $O/pmc_sel2 -o p -- python3 tools/select_bench.py --K 1000 --reps 1 > $O/pmc_sel2.log 2>&1 || return 7
  echo pmc-done
}

r4s1h() {
  # f3 selection: the LDS-tile kernel vs the direct-gather kernel (GMAGG_SELECT_DIRECT=1),
  # interleaved, plus the f3 parity tests on the direct kernel
  O=gpurun_out/r4s1h; mkdir -p $O
  GMAGG_SELECT_DIRECT=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_other_aggregators.py > $O/t_direct.log 2>&1 || { tail -30 $O/t_direct.log; return 1; }
  tail -1 $O/t_direct.log
  for r in 1 2; do
    for v in 0 1; do
      GMAGG_SELECT_DIRECT=$v timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 3 >> $O/select_direct$v.jsonl 2> $O/sel.err || return 2
    done
  done
  cat $O/select_direct*.jsonl
}

r4s1i() {
  # XCD placement of the resident grids: C2's 31 blocks on one XCD (GMAGG_RES_XCD=1),
  # the C5 groups numbered XCD by XCD (GMAGG_RB_XCD=1); parity first, then A/B
  O=gpurun_out/r4s1i; mkdir -p $O
  GMAGG_RES_XCD=1 GMAGG_RB_XCD=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_weiszfeld.py -k "resident or gm_host or philox or gm2_matches or clamp" > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 600 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant xcd=GMAGG_RES_XCD=1 --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -3 $O/ab_c2.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,0 --variant base= --variant xcd=GMAGG_RB_XCD=1 --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 3; }
  tail -3 $O/ab_c5air.log
  timeout -k 10 600 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant base= --variant xcd=GMAGG_RB_XCD=1 --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 4; }
  tail -3 $O/ab_c5.log
}

r4s1j() {
  # HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) of the C5 AirComp reading's
  # resident gm kernel, groups round-robin over the XCDs (base) vs numbered XCD by XCD
  O=gpurun_out/r4s1j; mkdir -p $O
  B="bench.py --workload c5 --reading aircomp --steps 1 --warmup 0 --no-cpu --alt-steps 0 --no-check --soak 0"
  for v in 0 1; do
    for c in FETCH_SIZE WRITE_SIZE; do
      GMAGG_RB_XCD=$v timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/x$v_$c -o p -- python3 $B > $O/x${v}_$c.log 2>&1 || return 1
      mv $O/x$v_$c $O/x${v}_$c
    done
    python3 tools/pmc_summary.py $O/x${v}_FETCH_SIZE/p_counter_collection.csv $O/x${v}_WRITE_SIZE/p_counter_collection.csv $O/pmc_x$v.json "c5 aircomp, GMAGG_RB_XCD=$v" > $O/summary_x$v.txt 2>&1 || return 2
    grep resident $O/summary_x$v.txt
  done
}

r4s1k() {
  # the batched resident kernel's poll back-off: s_sleep 1 (product) vs 4 (libgmagg_alt.so,
  # make alt ALT_FLAGS=-DGMK_RB_SLEEP=4): C5 AirComp throughput and exchange traffic
  O=gpurun_out/r4s1k; mkdir -p $O
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,0 --variant s1= --variant s4=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 1; }
  tail -2 $O/ab_c5air.log
  timeout -k 10 600 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant s1= --variant s4=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 2; }
  tail -2 $O/ab_c5.log
  B="bench.py --workload c5 --reading aircomp --steps 1 --warmup 0 --no-cpu --alt-steps 0 --no-check --soak 0"
  for c in FETCH_SIZE WRITE_SIZE; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/s4_$c -o p -- python3 $B > $O/s4_$c.log 2>&1 || return 3
  done
  python3 tools/pmc_summary.py $O/s4_FETCH_SIZE/p_counter_collection.csv $O/s4_WRITE_SIZE/p_counter_collection.csv $O/pmc_s4.json "c5 aircomp, sleep 4" > $O/summary_s4.txt 2>&1 || return 4
  grep resident $O/summary_s4.txt
}

r4s1l() {
  # the f3 selection's phases priced apart (K=1000 x 2M): product vs load-and-stage only
  # (libgmagg_sel1.so: -DGMK_SELECT_DBG=1) vs select on L2-resident tiles (sel2: DBG=2)
  O=gpurun_out/r4s1l; mkdir -p $O
  for r in 1 2; do
    for v in prod sel1 sel2; do
      lib=byzantine_aircomp_amd/libgmagg.so; [ $v != prod ] && lib=byzantine_aircomp_amd/libgmagg_$v.so
      GMAGG_LIB=$lib timeout -k 10 120 python -u tools/select_bench.py --K 1000 --reps 3 2> $O/err.log | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/phases.jsonl || return 1
    done
  done
  cat $O/phases.jsonl
}

r4s1m() {
  # the f3 selection's top byte (libgmagg_hist.so: -DGMK_SELECT_HIST=1) and top two bytes
  # (hist2: =2) from LDS histograms vs counting steps (product): parity of the f3 tests on
  # each, then interleaved timing
  O=gpurun_out/r4s1m; mkdir -p $O
  for v in hist hist2; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_other_aggregators.py > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; return 1; }
    tail -1 $O/t_$v.log
  done
  for r in 1 2; do
    for v in prod hist hist2; do
      lib=byzantine_aircomp_amd/libgmagg.so; [ $v != prod ] && lib=byzantine_aircomp_amd/libgmagg_$v.so
      GMAGG_LIB=$lib timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 3 2> $O/err.log | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/ab.jsonl || return 2
    done
  done
  cat $O/ab.jsonl
}

r4s1n() {
  # multi-rank rehearsals on one GPU after the round-4 changes: bench.py's N > 1 path
  # (torchrun, gloo, the torch all-reduce callback) for C3-small and for the whole C4 job
  # (d sharded in 2; the Gram guard decided on the all-reduced ||g||), then rank 0's
  # shard of an 8-GPU C4 job (its per-rank time before the cross-GPU all-reduce latency)
  O=gpurun_out/r4s1n; mkdir -p $O
  for w in c3-small c4; do
    timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --one-gpu --workload $w --no-cpu --alt-steps 0 --soak 0 --steps 3 --warmup 1 > $O/n2_$w.json 2> $O/n2_$w.err || { tail -20 $O/n2_$w.err; return 1; }
    cut -c1-900 $O/n2_$w.json
  done
  timeout -k 10 400 python -u bench.py --dist --rehearse-shard 8 --workload c4 --no-cpu --alt-steps 0 --soak 0 --steps 10 --warmup 2 > $O/c4_shard8.json 2> $O/c4_shard8.err || { tail -20 $O/c4_shard8.err; return 2; }
  cut -c1-900 $O/c4_shard8.json
}

r4s1o() {
  # round 4 session 1 closing set: GPU suite + smoke + the default bench line
  # (tools/final_check.sh), then every BASELINE workload's line and the f3 timings
  bash tools/final_check.sh || return $?
  O=gpurun_out/r4s1o; mkdir -p $O
  for w in "c2:--workload c2" "c5:--workload c5" "c5air:--workload c5 --reading aircomp" "c4:--workload c4 --steps 5 --warmup 1" "c4shard:--workload c4-shard"; do
    n=${w%%:*}; a=${w#*:}
    timeout -k 10 600 python -u bench.py $a > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; return 2; }
    cut -c1-300 $O/bench_$n.json
  done
  timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 3 > $O/select.jsonl 2> $O/select.err || return 3
  cat $O/select.jsonl
}

r4s2a() {
  # C2's single resident kernel with every block on one XCD AND the granules stored so that
  # they stay in that XCD's L2 (GMAGG_RES_XCD=2; the check-in confirms the placement from
  # XCC_ID, else agent-scope stores) against the default placement and the one-XCD placement
  # with agent-scope stores (=1, round 4: slower); parity of the resident tests first
  O=gpurun_out/r4s2a; mkdir -p $O
  GMAGG_RES_XCD=2 GMAGG_RES_VERBOSE=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_distributed.py -k "resident or gm_host or philox or gm2_matches or clamp" > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log; grep -c "local=1" $O/t.log; grep -c "local=0" $O/t.log
  GMAGG_RES_XCD=2 GMAGG_RES_VERBOSE=1 timeout -k 10 200 python -u bench.py --workload c2 --no-cpu --alt-steps 0 --soak 0 --steps 3 --warmup 1 > $O/c2_local.json 2> $O/c2_local.err || { tail -20 $O/c2_local.err; return 2; }
  sort $O/c2_local.err | uniq -c | head -5; cut -c1-400 $O/c2_local.json
  timeout -k 10 600 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant xcd1=GMAGG_RES_XCD=1 --variant local=GMAGG_RES_XCD=2 --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 3; }
  tail -4 $O/ab_c2.log
}

r4s2b() {
  # C5: whole groups per XCD with their granules kept in the XCD's L2 (GMAGG_RB_XCD=2)
  # against the XCD-major numbering (default, groups span 2-3 XCDs); parity first
  O=gpurun_out/r4s2b; mkdir -p $O
  GMAGG_RB_XCD=2 GMAGG_RES_VERBOSE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_c5_fullsize.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log; grep "resident_batched:" $O/t.log | sort | uniq -c | sort -rn | head -5
  GMAGG_RB_XCD=2 GMAGG_RES_VERBOSE=1 timeout -k 10 300 python -u bench.py --workload c5 --reading aircomp --no-cpu --alt-steps 0 --soak 0 --steps 1 --warmup 0 > $O/c5air_local.json 2> $O/c5air_local.err || { tail -20 $O/c5air_local.err; return 2; }
  sort $O/c5air_local.err | uniq -c | head -5; cut -c1-300 $O/c5air_local.json
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,0 --variant base= --variant local=GMAGG_RB_XCD=2 --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 3; }
  tail -3 $O/ab_c5air.log
  timeout -k 10 600 python -u tools/ab.py --rounds 3 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant base= --variant local=GMAGG_RB_XCD=2 --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 4; }
  tail -3 $O/ab_c5.log
}

r4s2c() {
  # C2 after the XCD-local exchange became the default: its exchange floor (libgmagg_alt.so
  # built with ALT_FLAGS=-DGMK_RES_DBG=7) in both exchange modes, the product at tol -1
  # (1000 iterations, same box), the resident / single-problem GPU tests, the kernel trace
  O=gpurun_out/r4s2c; mkdir -p $O
  B="--no-cpu --no-check --alt-steps 0 --soak 0"
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_training.py tests/test_gpu_distributed.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for m in 2 0; do
    GMAGG_RES_XCD=$m GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_exchange_only_x$m.json 2> $O/c2x$m.err || return 2
    GMAGG_RES_XCD=$m timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_tolneg_x$m.json 2> $O/c2_x$m.err || return 3
  done
  for f in $O/c2_*.json; do echo "$f $(python -c "import json,sys;l=json.load(open('$f'));print(l['ms_per_step'])")"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o t -- python3 bench.py --workload c2 --no-cpu --alt-steps 0 --soak 0 > $O/trace_c2.log 2>&1 || return 4
  head -4 $O/trace_c2/t_kernel_stats.csv
  timeout -k 10 200 python -u bench.py --workload c2 > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; return 5; }
  cut -c1-600 $O/bench_c2.json
}

r4s2d() {
  # C2 per-phase time of one iteration (block 0, s_memrealtime; libgmagg_alt.so built with
  # ALT_FLAGS=-DGMK_RES_PROF) with the XCD-local exchange (2) and the agent-scope one (0);
  # the local-vs-agent bit-identity test
  O=gpurun_out/r4s2d; mkdir -p $O
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py -k xcd_local > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for m in 2 0; do
    GMAGG_RES_XCD=$m GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 2 --warmup 1 --no-cpu --no-check --alt-steps 0 --soak 0 > $O/prof_x$m.json 2> $O/prof_x$m.err || return 2
    echo "mode $m"; grep GMK_RES_PROF $O/prof_x$m.err | tail -2
  done
}

r4s2e() {
  # C2 after the XCD-local exchange: the AirComp coefficients on v_rcp / v_rsq (fc:
  # libgmagg_alt_fc.so, -DGMK_RES_FASTCOEF=1), the gather in one round trip and one stage
  # (g1: libgmagg_alt_g1.so, -DGMK_RES_NBCHUNK=32), both (libgmagg_alt.so); parity of the
  # single-problem GPU tests on each, then interleaved A/B
  O=gpurun_out/r4s2e; mkdir -p $O
  for v in fc g1 both; do
    L=byzantine_aircomp_amd/libgmagg_alt_$v.so
    GMAGG_LIB=$L timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py > $O/t_$v.log 2>&1 || { tail -30 $O/t_$v.log; return 1; }
    echo "$L: $(tail -1 $O/t_$v.log)"
  done
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant fc=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_fc.so --variant g1=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_g1.so --variant both=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_both.so --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -5 $O/ab_c2.log
}

r4s2f() {
  # C5 AirComp: the column noise drawn one Philox block per 4 columns instead of one per
  # column (timing probe, different draws: libgmagg_alt_nz4.so, ALT_ONLY=resident_batched
  # ALT_FLAGS=-DGMK_RB_NZ4=1), interleaved A/B without the check
  O=gpurun_out/r4s2f; mkdir -p $O
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,0 --variant base= --variant nz4=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_nz4.so --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 1; }
  tail -3 $O/ab_c5air.log
}

r4s2g() {
  # single ClientPanels problems on C2's resident kernel (one XCD, panels read with the rows
  # tile): the panels / resident / weiszfeld GPU tests, C2 on panels vs rows, the training
  # loop (rows and panels)
  O=gpurun_out/r4s2g; mkdir -p $O
  timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_panels.py tests/test_gpu_resident_batched.py tests/test_gpu_weiszfeld.py tests/test_gpu_training.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 200 python -u bench.py --workload c2 --no-cpu --soak 0 > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; return 2; }
  python -c "import json;l=json.load(open('$O/c2.json'));print('c2', l['value'], l['ms_per_step'], json.dumps(l.get('alt_layout'))[:300])"
  timeout -k 10 300 python -u tools/loop_bench.py > $O/loop.jsonl 2> $O/loop.err || { tail -20 $O/loop.err; return 3; }
  cat $O/loop.jsonl
}

r4s2h() {
  # C2 poll tuning with the L2-kept exchange: no back-off between polls (s0: ALT_ONLY=resident
  # ALT_FLAGS=-DGMK_RES_SLEEP=0), 8 granules per round trip (c8: -DGMK_RES_NBCHUNK=8), both
  O=gpurun_out/r4s2h; mkdir -p $O
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_c8s0.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant s0=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_s0.so --variant c8=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_c8.so --variant c8s0=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_c8s0.so --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -4 $O/ab_c2.log
}

r4s2i() {
  # the median from a value-linear histogram (product: GMK_SELECT_VHIST=1) against the
  # bitwise selection (libgmagg_alt_novh.so: ALT_ONLY=coordinate ALT_FLAGS=-DGMK_SELECT_VHIST=0):
  # f3 parity on the product, then interleaved timing
  O=gpurun_out/r4s2i; mkdir -p $O
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_other_aggregators.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for r in 1 2; do
    for v in prod novh; do
      lib=byzantine_aircomp_amd/libgmagg.so; [ $v != prod ] && lib=byzantine_aircomp_amd/libgmagg_alt_$v.so
      GMAGG_LIB=$lib timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 3 2> $O/err.log | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/ab.jsonl || return 2
    done
  done
  cat $O/ab.jsonl
}

r4s2z() {
  # round 4 session 2 closing set: GPU suite + smoke + the default bench line
  # (tools/final_check.sh), every BASELINE workload's line, C2's kernel trace, the f3 timings
  bash tools/final_check.sh || return $?
  O=gpurun_out/r4s2z; mkdir -p $O
  for w in "c2:--workload c2" "c5:--workload c5" "c5air:--workload c5 --reading aircomp" "c4:--workload c4 --steps 5 --warmup 1" "c4shard:--workload c4-shard"; do
    n=${w%%:*}; a=${w#*:}
    timeout -k 10 600 python -u bench.py $a > $O/bench_$n.json 2> $O/bench_$n.err || { tail -20 $O/bench_$n.err; return 2; }
    cut -c1-300 $O/bench_$n.json
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o t -- python3 bench.py --workload c2 --no-cpu --alt-steps 0 --soak 0 > $O/trace_c2.log 2>&1 || return 3
  head -3 $O/trace_c2/t_kernel_stats.csv
  timeout -k 10 120 python -u tools/select_bench.py --K 1000 256 --reps 3 > $O/select.jsonl 2> $O/select.err || return 4
  cat $O/select.jsonl
}

r4s2j() {
  # f3 at K <= 1024 with one column per wave (GMAGG_SELECT_1COL=1: 54 VGPRs, 8 waves per
  # SIMD) against the column-pair kernel (4 waves per SIMD): parity, then interleaved timing
  O=gpurun_out/r4s2j; mkdir -p $O
  GMAGG_SELECT_1COL=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_other_aggregators.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for r in 1 2; do
    for v in 0 1; do
      GMAGG_SELECT_1COL=$v timeout -k 10 120 python -u tools/select_bench.py --K 1000 --reps 3 2> $O/err.log | sed "s/}$/, \"one_col\": $v}/" >> $O/ab.jsonl || return 2
    done
  done
  cat $O/ab.jsonl
}

r4s2k() {
  # f3 at K <= 256 with one column per wave (GMAGG_SELECT_1COL=2) against the column-pair
  # kernel: parity, then interleaved timing
  O=gpurun_out/r4s2k; mkdir -p $O
  GMAGG_SELECT_1COL=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_other_aggregators.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  for r in 1 2; do
    for v in -1 2; do
      GMAGG_SELECT_1COL=$v timeout -k 10 120 python -u tools/select_bench.py --K 256 --reps 3 2> $O/err.log | sed "s/}$/, \"one_col\": $v}/" >> $O/ab.jsonl || return 2
    done
  done
  cat $O/ab.jsonl
}

r4s2l() {
  # C5 AirComp draw placement (timing only, no check): the channel draw in draw_pass off
  # the critical path (eh: ALT_ONLY=resident_batched ALT_FLAGS=-DGMK_RB_EARLY_H2=1), one
  # Philox block per 4 columns (nz: -DGMK_RB_NZ4=1, different draws), both (ehnz)
  O=gpurun_out/r4s2l; mkdir -p $O
  timeout -k 10 1100 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,0 --variant base= --variant eh=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_eh.so --variant nz=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_nz.so --variant ehnz=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_ehnz.so --out $O/ab.jsonl > $O/ab.log 2>&1 || { tail -20 $O/ab.log; return 1; }
  tail -4 $O/ab.log
}

r4s2n() {
  # C2's resident tile: 16 waves x 4 rows (default) against 8 waves x 8 rows per lane
  # (GMAGG_RES_CFG=8,8: 512-thread blocks, half the waves in each reduction and barrier),
  # with 4 chunks per block (16 blocks, auto) or 2 (31 blocks); parity of the single-problem
  # tests on the 8-wave tile first
  O=gpurun_out/r4s2n; mkdir -p $O
  GMAGG_RES_CFG=8,8 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant w8=GMAGG_RES_CFG=8,8 --variant "w8c2=GMAGG_RES_CFG=8,8;GMAGG_RES_CPB=2" --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -3 $O/ab_c2.log
}

r4s2o() {
  # after C2's 8-wave resident tile became the default: the GPU suite + smoke + default bench,
  # C2's exchange floor on the new tile (libgmagg_alt.so: ALT_ONLY=resident
  # ALT_FLAGS=-DGMK_RES_DBG=7) and the product at tol -1, C2's bench line and kernel trace
  bash tools/final_check.sh || return $?
  O=gpurun_out/r4s2o; mkdir -p $O
  B="--no-cpu --no-check --alt-steps 0 --soak 0"
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_exchange_only.json 2> $O/c2x.err || return 2
  timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_tolneg.json 2> $O/c2.err || return 3
  for f in $O/c2_exchange_only.json $O/c2_tolneg.json; do echo "$f $(python -c "import json;print(json.load(open('$f'))['ms_per_step'])")"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c2 -o t -- python3 bench.py --workload c2 --no-cpu --alt-steps 0 --soak 0 > $O/trace_c2.log 2>&1 || return 4
  head -3 $O/trace_c2/t_kernel_stats.csv
  timeout -k 10 200 python -u bench.py --workload c2 > $O/bench_c2.json 2> $O/bench_c2.err || return 5
  cut -c1-300 $O/bench_c2.json
  timeout -k 10 300 python -u tools/loop_bench.py > $O/loop.jsonl 2> $O/loop.err || return 6
  head -2 $O/loop.jsonl | cut -c1-300
}

r4s2p() {
  # C2's resident tile, one step further: 4 waves of 16 rows (GMAGG_RES_CFG=4,16: 256-thread
  # blocks, one wave per SIMD) against the default 8 waves of 8; parity first
  O=gpurun_out/r4s2p; mkdir -p $O
  GMAGG_RES_CFG=4,16 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_panels.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant w4=GMAGG_RES_CFG=4,16 --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -2 $O/ab_c2.log
}

r4s2q() {
  # C2: wave 0 forms the coefficients right after summing the gathered values, one block
  # barrier fewer per iteration (libgmagg_alt_fuse.so: ALT_ONLY=resident
  # ALT_FLAGS=-DGMK_RES_FUSE_COEF=1); parity first
  O=gpurun_out/r4s2q; mkdir -p $O
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_fuse.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_panels.py tests/test_gpu_training.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant fuse=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_fuse.so --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -2 $O/ab_c2.log
}

r4s2r() {
  # C2's HBM traffic per launch (FETCH_SIZE / WRITE_SIZE, one counter per pass) with the
  # L2-kept exchange (default) and with agent-scope stores over every XCD (GMAGG_RES_XCD=0);
  # then the multi-rank rehearsals of r4s1n on the final code
  O=gpurun_out/r4s2r; mkdir -p $O; export TMPDIR=/tmp
  B="bench.py --workload c2 --steps 3 --warmup 1 --no-cpu --alt-steps 0 --no-check --soak 0"
  for v in 2 0; do
    for c in FETCH_SIZE WRITE_SIZE; do
      GMAGG_RES_XCD=$v timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $O/x${v}_$c -o p -- python3 $B > $O/x${v}_$c.log 2>&1 || return 1
    done
    python3 tools/pmc_summary.py $O/x${v}_FETCH_SIZE/p_counter_collection.csv $O/x${v}_WRITE_SIZE/p_counter_collection.csv $O/pmc_x$v.json "c2 rows, GMAGG_RES_XCD=$v" > $O/summary_x$v.txt 2>&1 || return 2
    grep -i resident $O/summary_x$v.txt | head -3
  done
  bash tools/gpu_sets.sh r4s1n
}

r4s2s() {
  # C5: the batched kernel's AirComp coefficients on v_rcp / v_rsq (fc: ALT_ONLY=
  # resident_batched ALT_FLAGS=-DGMK_RB_FASTCOEF=1) on the AirComp reading; the OMA pre-noise
  # drawn 4 (oma4) or 1 (oma1) rows at a time instead of 2 on the prenoise reading
  O=gpurun_out/r4s2s; mkdir -p $O
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_fc.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py tests/test_gpu_c5_fullsize.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--reading,aircomp,--no-cpu,--alt-steps,0,--soak,0,--no-check,--steps,1,--warmup,0 --variant base= --variant fc=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_fc.so --out $O/ab_c5air.jsonl > $O/ab_c5air.log 2>&1 || { tail -20 $O/ab_c5air.log; return 2; }
  tail -2 $O/ab_c5air.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant base= --variant oma4=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_oma4.so --variant oma1=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_oma1.so --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 3; }
  tail -3 $O/ab_c5.log
}

r4s2t() {
  # C5 prenoise: the OMA pre-noise drawn 4 (oma4) or 1 (oma1) rows at a time instead of 2
  O=gpurun_out/r4s2t; mkdir -p $O
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_oma4.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_resident_batched.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 2 --bench=--workload,c5,--no-cpu,--alt-steps,0,--soak,0,--no-check --variant base= --variant oma4=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_oma4.so --variant oma1=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_oma1.so --out $O/ab_c5.jsonl > $O/ab_c5.log 2>&1 || { tail -20 $O/ab_c5.log; return 3; }
  tail -3 $O/ab_c5.log
}

r4s2u() {
  # C2's grid: 3 chunks per block (GMAGG_RES_CPB=3: 21 blocks of 384 columns) against 2
  # (31 blocks, default); parity on it first
  O=gpurun_out/r4s2u; mkdir -p $O
  GMAGG_RES_CPB=3 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py -k "golden or gm_ or resident" > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant cpb3=GMAGG_RES_CPB=3 --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -2 $O/ab_c2.log
}

r4s2v() {
  # C2's grid: 1 chunk per block, 62 blocks, two per CU of the one XCD (GMAGG_RES_CPB=1
  # GMAGG_RES_XCD_BPC=2) against 2 chunks per block (31 blocks, default)
  O=gpurun_out/r4s2v; mkdir -p $O
  GMAGG_RES_CPB=1 GMAGG_RES_XCD_BPC=2 GMAGG_RES_VERBOSE=1 timeout -k 10 200 python -u bench.py --workload c2 --no-cpu --alt-steps 0 --soak 0 --steps 3 --warmup 1 > $O/c2_b2.json 2> $O/c2_b2.err || { tail -20 $O/c2_b2.err; return 1; }
  sort $O/c2_b2.err | uniq -c | head -4; cut -c1-200 $O/c2_b2.json
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base= --variant "b2=GMAGG_RES_CPB=1;GMAGG_RES_XCD_BPC=2" --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -2 $O/ab_c2.log
}

r4s2w() {
  # C2: thread 0's movement / ||g||^2 partial sums hoisted before phase B (product) against
  # the previous kernel (libgmagg_alt_base.so: HEAD's resident.hip); parity first
  O=gpurun_out/r4s2w; mkdir -p $O
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_weiszfeld.py tests/test_gpu_panels.py > $O/t.log 2>&1 || { tail -30 $O/t.log; return 1; }
  tail -1 $O/t.log
  timeout -k 10 900 python -u tools/ab.py --rounds 3 --bench=--workload,c2,--no-cpu,--alt-steps,0,--soak,0 --variant base=GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_base.so --variant fin= --out $O/ab_c2.jsonl > $O/ab_c2.log 2>&1 || { tail -20 $O/ab_c2.log; return 2; }
  tail -2 $O/ab_c2.log
}

r4s2y() {
  # kernel traces (rocprofv3 --kernel-trace --stats) of the default bench line (C3) and of the
  # C5 and C4 lines on the final code, to pair each line's HIP-event timing with rocprof
  O=gpurun_out/r4s2y; mkdir -p $O; export TMPDIR=/tmp
  B="--no-cpu --alt-steps 0 --soak 0"
  for w in "c3:" "c5:--workload c5" "c4:--workload c4 --steps 3 --warmup 1"; do
    n=${w%%:*}; a=${w#*:}
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_$n -o t -- python3 bench.py $a $B > $O/trace_$n.json 2> $O/trace_$n.err || return 1
    head -4 $O/trace_$n/t_kernel_stats.csv | cut -c1-200
    python3 -c "import json;l=json.load(open('$O/trace_$n.json'));print('$n bench avg_launch_us', l['roofline'].get('avg_launch_us'))"
  done
}

r4s2x() {
  # the single-problem resident kernel beyond C2's shape: the default 8-wave tile against the
  # previous 16-wave one (GMAGG_RES_CFG=16,4), at d = 7,850 (one XCD), 20,000 and 48,670
  # (the EMNIST MLP: grids too large for one XCD)
  O=gpurun_out/r4s2x; mkdir -p $O
  for r in 1 2; do
    for v in default 16,4; do
      if [ $v = default ]; then e=""; else e="GMAGG_RES_CFG=$v"; fi
      env $e timeout -k 10 300 python -u tools/res_shape_bench.py >> $O/shapes.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 1; }
    done
  done
  cat $O/shapes.jsonl
}

r4s2aa() {
  # the resident kernel's gather at large grids: 8 or 16 granules per poll round trip
  # (libgmagg_alt_c8.so / _c16.so: ALT_ONLY=resident ALT_FLAGS=-DGMK_RES_NBCHUNK=8 / 16)
  # against 4, at d = 7,850 / 20,000 / 48,670
  O=gpurun_out/r4s2aa; mkdir -p $O
  for r in 1 2; do
    for v in base c8 c16; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt_$v.so"
      env $L timeout -k 10 300 python -u tools/res_shape_bench.py --shapes 50x7850,50x20000,50x48670 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/shapes.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 1; }
    done
  done
  cat $O/shapes.jsonl | cut -c1-120
}

r4s3a() {
  # the client chain (clients.hip): dz in dynamic LDS so the reference's B = 50 tile is
  # staged (product: + the next client's tile prefetched behind phases B / C) against
  # libgmagg_nopf.so (staged, no prefetch) and libgmagg_old.so (the previous kernel: B = 50
  # not staged); then the phase probes (-DGMK_CC_PROF: _prof, _prof0, _profold)
  O=gpurun_out/r4s3a; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2; do
    for v in base nopf old; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
  for v in prof prof0 profold; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so timeout -k 10 300 python -u tools/loop_bench.py --steps 5 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; return 3; }
    grep GMK_CC_PROF $O/$v.log | tail -3
  done
  cut -c1-60,150-260 $O/loop.jsonl
}

r4s3b() {
  # the client chain: the product (staged B = 50 tile, bias in LDS, phase A's groups
  # unrolled; the loop draws the next step's indices while the GPU runs) against
  # libgmagg_nounroll.so (-DGMK_CC_UNROLL_A=0), _nopf (r4s3a's staged kernel) and _old (the
  # kernel before r4s3a); the phase probe (-DGMK_CC_PROF)
  O=gpurun_out/r4s3b; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2; do
    for v in base nounroll nopf old; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
  for v in prof; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so timeout -k 10 300 python -u tools/loop_bench.py --steps 5 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; return 3; }
    grep GMK_CC_PROF $O/$v.log | tail -3
  done
  cut -c1-60,150-260 $O/loop.jsonl
}

r4s3c() {
  # the client chain: phase A's tile loads unconditional at clamped addresses, masked after
  # (product) against libgmagg_noclamp.so (-DGMK_CC_CLAMP=0: per-load branches, a wait per
  # row), _s3b (r4s3b's product) and _old (before r4s3a); phase probes _prof / _profnc
  O=gpurun_out/r4s3c; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2; do
    for v in base noclamp s3b old; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
  for v in prof profnc; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so timeout -k 10 300 python -u tools/loop_bench.py --steps 5 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; return 3; }
    grep GMK_CC_PROF $O/$v.log | tail -3
  done
  cut -c1-60,150-260 $O/loop.jsonl
}

r4s3z() {
  # round 4 session 3 closing set: GPU suite + smoke + the default bench line
  # (tools/final_check.sh), the training loop (product library) and its kernel trace
  bash tools/final_check.sh || return $?
  O=gpurun_out/r4s3z; mkdir -p $O
  timeout -k 10 300 python -u tools/loop_bench.py --steps 20 > $O/loop.jsonl 2> $O/loop.err || { tail -20 $O/loop.err; return 2; }
  cut -c1-60,150-260 $O/loop.jsonl
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_loop -o t -- python3 tools/loop_bench.py --steps 20 > $O/trace_loop.log 2>&1 || return 3
  head -4 $O/trace_loop/t_kernel_stats.csv
}

r4s3d() {
  # the client chain's phase A as float2 loads when F is even (product) against
  # libgmagg_v1.so (-DGMK_CC_V2=0: the scalar slots); phase probes _prof / _prof1
  O=gpurun_out/r4s3d; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2 3; do
    for v in base v1; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
  for v in prof prof1; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so timeout -k 10 300 python -u tools/loop_bench.py --steps 5 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; return 3; }
    grep GMK_CC_PROF $O/$v.log | tail -2
  done
}

r4s3e() {
  # the client chain's phase A reading W from LDS (copied once per client; product) against
  # libgmagg_nowl.so (-DGMK_CC_WLDS=0: every wave loads the W columns from global memory);
  # phase probes _prof / _profnw
  O=gpurun_out/r4s3e; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2 3; do
    for v in base nowl; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
  for v in prof profnw; do
    GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so timeout -k 10 300 python -u tools/loop_bench.py --steps 5 > $O/$v.log 2>&1 || { tail -20 $O/$v.log; return 3; }
    grep GMK_CC_PROF $O/$v.log | tail -2
  done
}

r4s3f() {
  # the client chain's next row / label loaded during phase C (product) against
  # libgmagg_head.so (the setup's two dependent loads per client)
  O=gpurun_out/r4s3f; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2 3; do
    for v in base head; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
}

# (r4s3d-r4s3g: A/B sets of variants that were measured and not kept; their knobs are no
# longer in clients.hip — DESIGN.md §3.5 records each result)
r4s3g() {
  # the client chain's logits on f32 MFMA (product) against libgmagg_nomf.so
  # (-DGMK_CC_MFMA=0: the VALU dots); phase probe _prof
  O=gpurun_out/r4s3g; mkdir -p $O
  timeout -k 10 400 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; return 1; }
  tail -2 $O/tests.log
  for r in 1 2 3; do
    for v in base nomf; do
      L=""; [ $v != base ] && L="GMAGG_LIB=byzantine_aircomp_amd/libgmagg_$v.so"
      env $L timeout -k 10 300 python -u tools/loop_bench.py --steps 20 | sed "s/}$/, \"lib\": \"$v\"}/" >> $O/loop.jsonl 2> $O/err.log || { tail -20 $O/err.log; return 2; }
    done
  done
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_prof.so timeout -k 10 300 python -u tools/loop_bench.py --steps 5 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; return 3; }
  grep GMK_CC_PROF $O/prof.log | tail -2
}

[ $# -eq 1 ] && declare -F "$1" > /dev/null || { echo "usage: $0 SET  (sets: $(declare -F | awk '{print $3}' | tr '\n' ' '))"; exit 2; }
"$1"
