# Closing-pass (mode 3) and STEP-pass tile sweep at K=256 (C4 shard): rocprof averages.
set -o pipefail
mkdir -p gpurun_out/sweep_close
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in ${CFGS:-16,32,8,1 16,64,16,1}; do
  tag=$(echo $cfg | tr , _)
  GMAGG_PASS_CFG=$cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep_close/$tag -o s -- python3 bench.py --workload c4-shard --algo gram --steps 4 --warmup 1 --no-cpu > gpurun_out/sweep_close/$tag.log 2>&1 || { echo "fail $cfg"; tail -5 gpurun_out/sweep_close/$tag.log; exit 1; }
  GMAGG_PASS_CFG=$cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/sweep_close/st$tag -o s -- python3 bench.py --workload c4-shard --algo stream --steps 2 --warmup 1 --no-cpu > gpurun_out/sweep_close/st$tag.log 2>&1 || { echo "fail stream $cfg"; exit 1; }
  python3 - "$cfg" "$tag" <<'PY'
import csv,sys,glob
cfg,tag=sys.argv[1],sys.argv[2]
def get(d):
    f=glob.glob(f'gpurun_out/sweep_close/{d}/**/s_kernel_stats.csv',recursive=True)[0]
    out={}
    for r in csv.DictReader(open(f)):
        if 'weiszfeld_pass' in r['Name']:
            mode=r['Name'].split('<')[1].split(',')[4].strip()
            out[mode]=float(r['AverageNs'])/1e3
    return out
a=get(tag); b=get('st'+tag)
print(cfg, 'close(mode3) us', a.get('3'), 'step(mode0) us', b.get('0'), 'init(mode1) us', b.get('1'))
PY
done
