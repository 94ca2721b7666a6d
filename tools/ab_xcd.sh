# A/B of the XCD run length (ORBHIP_XCD_RUN) on one box: C2 headline + in-flight + C3 rate.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python3 -m pytest tests/test_extract_gpu.py tests/test_c3_batch_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { tail -5 gpurun_out/ab_tests.log; exit 1; }
for xr in ${RUNS:-0 16 0 16}; do
  ORBHIP_XCD_RUN=$xr timeout -k 10 300 python3 bench.py --no-cpu --extra-timeout 200 > gpurun_out/ab_$xr.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/ab_$xr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); e=d['extra']; print('xrun=$xr', d['value'], d['batch1_latency_ms'], d['config']['one_camera_8_in_flight_frames_per_s'], 'c3', e.get('c3_1280x720_b64_extract_match_frames_per_s'), e.get('c3_roofline',{}).get('stage_avg_ms'))"
done
