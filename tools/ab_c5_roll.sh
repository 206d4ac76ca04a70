# A/B: C5 batched sweep, plain pass (default for row-major input) vs rolling prefetch.
set -o pipefail
mkdir -p gpurun_out/c5ab
timeout -k 10 300 python -u tools/sweep_c5.py > gpurun_out/c5ab/plain.jsonl 2> gpurun_out/c5ab/plain.err || exit 1
GMAGG_PASS_VARIANT=2 timeout -k 10 300 python -u tools/sweep_c5.py > gpurun_out/c5ab/roll.jsonl 2> gpurun_out/c5ab/roll.err || exit 2
timeout -k 10 300 python -u tools/sweep_c5.py > gpurun_out/c5ab/plain2.jsonl 2> gpurun_out/c5ab/plain2.err || exit 3
for f in plain roll plain2; do echo $f; cut -c1-200 gpurun_out/c5ab/$f.jsonl; done
