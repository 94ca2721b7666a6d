# C2 pipelined rate vs HIP hardware queues per process and frames in flight.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for q in 4 8; do for s in 4 6 8; do GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu --no-extra --inflight $s 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('queues=$q inflight=$s', d['value'], c['sequential_frames_per_s'], c['host_submit_ms_per_frame'])"; done; done
