set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/multi_thread_c2.py 300 > gpurun_out/mt.log 2>&1 || exit 1
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu --no-extra --steps 200 > gpurun_out/q_$q.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/q_$q.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('queues=$q', d['value'], d['batch1_frames_per_s'], c['host_submit_ms_per_frame'])"
done
grep -v amdgpu mt.log 2>/dev/null; cat gpurun_out/mt.log | grep -v amdgpu
