set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2f; mkdir -p $o
for dbg in 0 1 2 4 8 16 31; do
  GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so GMAGG_RB_DBG=$dbg timeout -k 10 200 python -u tools/rb_probe.py --quick > $o/dbg$dbg.log 2>&1 || { tail -5 $o/dbg$dbg.log; exit 1; }
  grep fit $o/dbg$dbg.log
done
