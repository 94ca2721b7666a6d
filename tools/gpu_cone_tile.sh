# C2 16-camera headline and batch-1 per cone tile edge (ORBHIP_CONE_TILE overrides the front-end's 14).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for ts in ${TILES:-10 12 14 16 20}; do
  ORBHIP_CONE_TILE=$ts timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra --steps 300 > gpurun_out/cone_tile.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/cone_tile.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('tile $ts', d['value'], d['batch1_frames_per_s'])"
done
