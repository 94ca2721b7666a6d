# C3 k_fast_cells time per threads-per-cell choice (ORBHIP_FAST_NT).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for nt in ${NTS:-256 128 512}; do
  ORBHIP_FAST_NT=$nt timeout -k 10 300 python3 -u bench.py --no-cpu --steps 100 > gpurun_out/fastnt.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/fastnt.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('nt=$nt', 'C2', d['value'], 'C3', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_roofline']['stage_avg_ms']['k_fast_cells'])"
done
