# Round 2: K=256 closing/STEP tile A/B on panels: (16,32,8,OCC1) vs (8,32,16,OCC2) (same
# J = 128 columns = the panel width), C4 shard aggregation interleaved, + kernel traces.
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/r2r
mkdir -p $O
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > $O/$name.log 2>&1
  local rc=$?
  echo "[$name] rc=$rc"; tail -1 $O/$name.log | cut -c1-200
  if [ $rc -ne 0 ]; then exit $rc; fi
  return 0
}
step tests 300 python -u -m pytest tests/test_gpu_panels.py -q -x --timeout 120 --timeout-method thread
cd /tmp && export TMPDIR=/tmp
B="$GRAFT_REPO_ROOT/bench.py --workload c4-shard --steps 10 --warmup 2 --no-cpu --alt-steps 0 --no-check"
for v in a b a2 b2; do
  case $v in a*) cfg="";; b*) cfg="8,32,16,2";; esac
  GMAGG_PASS_CFG=$cfg step ab_$v 200 python3 $B
  echo "$v cfg=$cfg $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*\|"gram_guard": "[a-z]*"' $O/ab_$v.log | tr '\n' ' ')"
done
for v in a b; do
  case $v in a*) cfg="";; b*) cfg="8,32,16,2";; esac
  GMAGG_PASS_CFG=$cfg step kt_$v 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o run -- python3 $B
  python3 $GRAFT_REPO_ROOT/tools/trace_summary.py $O/kt_$v/run_kernel_trace.csv | grep -E "weiszfeld_pass|gram_h16" | cut -c1-120
done
# the same tile for a K=256 streaming gm2 (algo=stream) on panels
for v in a b; do
  case $v in a*) cfg="";; b*) cfg="8,32,16,2";; esac
  GMAGG_PASS_CFG=$cfg step st_$v 200 python3 $B --algo stream
  echo "stream $v $(grep -o '"avg_launch_us": [0-9.]*\|"ms_per_step": [0-9.]*' $O/st_$v.log | tr '\n' ' ')"
done
