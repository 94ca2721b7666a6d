# C2 pipelined rate vs frames in flight (+ the pipelined-stream parity test first).
cd "${GRAFT_REPO_ROOT:-/root/repo}"
timeout -k 10 300 python -u -m pytest tests/test_bench_stream.py -x -q -m gpu --timeout 200 --timeout-method thread 2>&1 | tail -2 || exit 1
for s in 1 4 6 8 12; do timeout -k 10 200 python bench.py --no-cpu --no-extra --inflight $s 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('inflight=$s', d['value'], c['sequential_frames_per_s'], c['host_submit_ms_per_frame'], c['matches_last_pair'])"; done
