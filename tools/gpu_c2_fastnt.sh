# C2 16-camera headline and batch-1 per FAST threads-per-cell override (ORBHIP_FAST_NT).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for nt in default 256 1024; do
  if [ $nt = default ]; then unset ORBHIP_FAST_NT; else export ORBHIP_FAST_NT=$nt; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra --steps 300 > gpurun_out/nt2.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/nt2.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('nt $nt', d['value'], d['batch1_frames_per_s'])"
done
