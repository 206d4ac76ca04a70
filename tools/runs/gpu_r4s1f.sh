# Round 4 session 1: latency-roofline probes (exchange floor, VALU instruction counts)
# and the whole-C4 Gram job's trace + PMC traffic.
set -o pipefail
O=gpurun_out/r4s1f; mkdir -p $O; export TMPDIR=/tmp
B="--no-cpu --no-check --alt-steps 0 --soak 0"
GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_exchange_only.json 2> $O/c2x.err || exit 2
timeout -k 10 200 python -u bench.py --workload c2 --tol -1 --steps 5 $B > $O/c2_tolneg.json 2> $O/c2.err || exit 3
for w in "c2:--workload c2 --steps 3" "c5air:--workload c5 --reading aircomp --steps 1 --warmup 0" "c5pre:--workload c5 --steps 1 --warmup 0"; do
  n=${w%%:*}; a=${w#*:}
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES --output-format csv -d $O/pmc_valu_$n -o p -- python3 bench.py $a $B > $O/pmc_valu_$n.log 2>&1 || exit 4
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_c4 -o t -- python3 bench.py --workload c4 --steps 3 --warmup 1 $B > $O/trace_c4.log 2>&1 || exit 5
head -5 $O/trace_c4/t_kernel_stats.csv
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 400 rocprofv3 --pmc $c --output-format csv -d $O/pmc_c4_$c -o p -- python3 bench.py --workload c4 --steps 2 --warmup 1 $B > $O/pmc_c4_$c.log 2>&1 || exit 6
done
ls -R $O | head -40
