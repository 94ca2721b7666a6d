# Matcher (fused / two-kernel), launch-graph replay and pipelined-stream parity, then the C2 trace
# and an A/B of the one-launch matcher in the C2 bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_match_gpu.py tests/test_extract_gpu.py tests/test_bench_stream.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/g_tests.log 2>&1; rc=$?; tail -5 gpurun_out/g_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/trace_c2.py 2>&1 | grep -v amdgpu.ids && \
for u in 0 1; do ORBHIP_MATCH_UNFUSED=$u timeout -k 10 200 python bench.py --no-cpu --no-extra 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('unfused=$u', d['value'], c['sequential_frames_per_s'], c['host_submit_ms_per_frame'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"; done
