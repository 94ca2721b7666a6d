# r05: device trace of one C2 step (per-kernel spans, octree level-0 phase cycles), three frames
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_octtrace
mkdir -p $O
for b in 0 0; do
  ORBHIP_TRACE_BLOCK=$b timeout -k 10 180 python3 -u tools/trace_c2.py > $O/trace_$b.log 2>&1 || { tail -20 $O/trace_$b.log; exit 1; }
  grep -v amdgpu.ids $O/trace_$b.log
done
