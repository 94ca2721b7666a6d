cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2; do
for g in 0 1; do ORBHIP_NO_GRAPH=$g timeout -k 10 200 python bench.py --no-cpu --no-extra 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('no_graph=$g', d['value'], c['sequential_frames_per_s'], c['host_submit_ms_per_frame'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"; done
done
