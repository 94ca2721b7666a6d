cd "${GRAFT_REPO_ROOT:-/root/repo}"
for s in 1 2 3 4 6; do timeout 200 python bench.py --no-cpu --no-extra --steps 600 --inflight $s 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($s, d['value'], d['config']['sequential_frames_per_s'], d['config']['matches_last_pair'], d['roofline']['avg_launch_ms'])"; done
