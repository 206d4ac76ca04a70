set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
o=gpurun_out/r3s2i; mkdir -p $o
timeout -k 10 300 python -u tools/rb_probe.py > $o/cur.log 2>&1 || { tail -5 $o/cur.log; exit 1; }
GMAGG_LIB=byzantine_aircomp_amd/libgmagg_alt.so timeout -k 10 300 python -u tools/rb_probe.py > $o/old.log 2>&1 || { tail -5 $o/old.log; exit 1; }
echo cur; grep fit $o/cur.log; echo old; grep fit $o/old.log
