# C2 16-camera headline vs HIP hardware queues per process (GPU_MAX_HW_QUEUES) and camera count.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for q in 4 8 16 4 8 16; do for c in 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu --no-extra --cameras $c --steps 200 > gpurun_out/q_$q.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/q_$q.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('queues=$q cameras=$c', d['value'], d['batch1_frames_per_s'], c['host_submit_ms_per_frame'])"
done; done
