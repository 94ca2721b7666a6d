# C2 single-frame chain after a kernel change: extract / match / projection parity, the device
# phase trace of one frame (tools/trace_c2.py, work-group 0), and the C2 bench section
# (16-camera value, one-camera batch-1 latency, stage averages).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c2chain
timeout -k 10 400 python3 -u -m pytest tests/test_extract_gpu.py tests/test_match_gpu.py tests/test_frontend.py tests/test_projection.py -m gpu -x -q \
    --timeout 240 --timeout-method thread > gpurun_out/c2chain/pytest.log 2>&1 || { tail -30 gpurun_out/c2chain/pytest.log; exit 1; }
tail -1 gpurun_out/c2chain/pytest.log
ORBHIP_TRACE_BLOCK=0 timeout -k 10 120 python3 -u tools/trace_c2.py > gpurun_out/c2chain/trace.log 2>&1 || { tail gpurun_out/c2chain/trace.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c2chain/trace.log
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --no-cpu --no-extra > gpurun_out/c2chain/bench$i.log 2>&1 || { tail gpurun_out/c2chain/bench$i.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/c2chain/bench$i.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('value', d['value'], 'batch1_ms', d['batch1_latency_ms'], r['kernel'], r['avg_launch_ms'])
print('stages', r['stage_avg_ms']); print('one-frame stages', r.get('stage_avg_ms_one_frame_stream'))"
done
