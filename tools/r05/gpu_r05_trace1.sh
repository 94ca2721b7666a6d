# r05: one C2 device trace (octree / cone phase cycles of work-group 0)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_trace1
mkdir -p $O
for i in 1 2; do
  ORBHIP_TRACE_BLOCK=0 timeout -k 10 180 python3 -u tools/trace_c2.py > $O/trace_$i.log 2>&1 || { tail -20 $O/trace_$i.log; exit 1; }
  grep -A2 "k_octree\|k_pyr_cone" $O/trace_$i.log | grep -v "per-wg"
done
