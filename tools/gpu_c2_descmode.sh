# C2 16-camera headline and batch-1 with the descriptor kernel per keypoint-work-group (default
# at one frame) vs a wave per keypoint (ORBHIP_DESC_MODE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for m in default 0; do
  if [ $m = default ]; then unset ORBHIP_DESC_MODE; else export ORBHIP_DESC_MODE=$m; fi
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra --steps 300 > gpurun_out/dm.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/dm.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('desc_mode $m', d['value'], d['batch1_frames_per_s'])"
done
