# C5 tile sweep (batched K=50 x d=100k): the default (16,64,4) vs two-blocks-per-CU tiles.
set -o pipefail
mkdir -p gpurun_out/c5t
for cfg in default 16,64,4,2 8,32,4 16,32,8,2 default; do
  if [ $cfg = default ]; then unset GMAGG_PASS_CFG; else export GMAGG_PASS_CFG=$cfg; fi
  timeout -k 10 200 python -u tools/sweep_c5.py --problems 2048 > gpurun_out/c5t/$cfg.jsonl 2> gpurun_out/c5t/$cfg.err || { tail -5 gpurun_out/c5t/$cfg.err; exit 1; }
  python3 -c "
import json
L=[json.loads(l) for l in open('gpurun_out/c5t/$cfg.jsonl')]
print('$cfg', ' '.join('%s=%.0fGB/s'%(l['var'],l['GBps_streamed']) for l in L if 'var' in l), 'total_s=%.2f'%L[-1]['seconds'])"
done
