#!/bin/bash
# One parameterised GPU-box runner (replaces the round-2 one-off gpu_r2*.sh scripts).
#
#   bash tools/gpu.sh TAG STEP [STEP ...]
#
# Output goes to gpurun_out/TAG/.  Each STEP runs under its own time limit; the
# script stops at the first failing step (nothing more runs on the GPU after a
# fault, an abort or a timeout).  STEP forms:
#   suite[:PYTEST_ARGS]       pytest -m gpu (all tests, or the given files / -k args)
#   smoke                     __graft_entry__.smoke()
#   bench:NAME[:ARGS]         python bench.py ARGS  -> NAME.json / NAME.err
#   trace:NAME[:ARGS]         rocprofv3 --kernel-trace --stats of bench.py ARGS -> NAME/
#   pmc:NAME:COUNTER[:ARGS]   one rocprofv3 --pmc pass (one counter) of bench.py ARGS
#   py:NAME:SCRIPT[:ARGS]     python SCRIPT ARGS -> NAME.log (tools/*.py probes)
#   run:NAME:CMD              a built probe binary (tools/*.hip) -> NAME.log
#   env:VAR=VALUE             export for the following steps
set -o pipefail
tag=$1
shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd "${GRAFT_REPO_ROOT:-.}" || exit 9
for step in "$@"; do
  kind=${step%%:*}
  rest=${step#*:}
  [ "$rest" = "$step" ] && rest=""
  echo "== $step" >&2
  case $kind in
    env)
      export "$rest"
      ;;
    suite)
      timeout -k 10 900 python -u -m pytest -m gpu -q -x --timeout 120 --timeout-method thread \
        ${rest:-tests} > "$out/pytest_gpu.log" 2>&1
      rc=$?; tail -3 "$out/pytest_gpu.log"
      if [ $rc -ne 0 ]; then
        grep -E "^(FAILED|ERROR)|Error|assert" "$out/pytest_gpu.log" | head -20; exit $rc
      fi
      ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 \
        || { tail -20 "$out/smoke.log"; exit 2; }
      grep smoke "$out/smoke.log"
      ;;
    bench)
      name=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      timeout -k 10 900 python -u bench.py $args > "$out/$name.json" 2> "$out/$name.err" \
        || { rc=$?; tail -20 "$out/$name.err"; exit $rc; }
      cat "$out/$name.json"
      ;;
    trace)
      name=${rest%%:*}; args=${rest#*:}; [ "$args" = "$rest" ] && args=""
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$name" -o t -- \
        python3 bench.py $args > "$out/$name.log" 2>&1 || { rc=$?; tail -30 "$out/$name.log"; exit $rc; }
      head -6 "$out/$name/t_kernel_stats.csv"
      ;;
    pmc)
      name=${rest%%:*}; r2=${rest#*:}; ctr=${r2%%:*}; args=${r2#*:}; [ "$args" = "$r2" ] && args=""
      timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d "$out/$name" -o p -- \
        python3 bench.py $args > "$out/$name.log" 2>&1 || { rc=$?; tail -20 "$out/$name.log"; exit $rc; }
      ;;
    py)
      name=${rest%%:*}; r2=${rest#*:}; script=${r2%%:*}; args=${r2#*:}; [ "$args" = "$r2" ] && args=""
      timeout -k 10 900 python -u "$script" $args > "$out/$name.log" 2>&1 \
        || { rc=$?; tail -30 "$out/$name.log"; exit $rc; }
      tail -40 "$out/$name.log"
      ;;
    run)
      name=${rest%%:*}; cmd=${rest#*:}
      timeout -k 10 600 $cmd > "$out/$name.log" 2>&1 || { rc=$?; tail -30 "$out/$name.log"; exit $rc; }
      tail -40 "$out/$name.log"
      ;;
    *)
      echo "unknown step $step" >&2; exit 8
      ;;
  esac
done
