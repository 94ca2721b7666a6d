# C2 section under 4 (the box default), 8 and 16 hardware queues per process: the 16 camera
# streams share the process's hardware queues, so this measures what that sharing costs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/hwq
for q in 4 16 8 4 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra > gpurun_out/hwq/q$q.log 2>&1 || { tail gpurun_out/hwq/q$q.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/hwq/q$q.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('hwq $q value', d['value'], 'batch1_ms', d['batch1_latency_ms'], r['kernel'], r['avg_launch_ms'])
print('  stages', r['stage_avg_ms'])"
done
