# Front-end stream parity on the GPU, then the C2 bench across frames in flight.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_frontend.py tests/test_bench_stream.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/fe_tests.log 2>&1; rc=$?; tail -15 gpurun_out/fe_tests.log; [ $rc -eq 0 ] || exit $rc
for s in 4 8 12 16; do timeout -k 10 200 python bench.py --no-cpu --no-extra --inflight $s 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('inflight=$s', d['value'], c['sequential_frames_per_s'], c['host_submit_ms_per_frame'], c['matches_last_pair'], c['keypoints_per_frame'], d['roofline']['kernel'])"; done
