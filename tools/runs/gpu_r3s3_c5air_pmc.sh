#!/bin/bash
# HBM traffic of the C5 AirComp reading's resident gm kernel: FETCH_SIZE and WRITE_SIZE,
# each in its own pass, then tools/pmc_summary.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/c5air_pmc
mkdir -p $O
B="bench.py --workload c5 --reading aircomp --steps 1 --warmup 0 --no-cpu --alt-steps 0 --no-check"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/f -o p -- python3 $B > $O/f.json 2> $O/f.err &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/w -o p -- python3 $B > $O/w.json 2> $O/w.err &&
python3 tools/pmc_summary.py $O/f/p_counter_collection.csv $O/w/p_counter_collection.csv $O/pmc.json "c5 aircomp reading, panels, resident" > $O/summary.txt 2>&1
