set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cm in 1024 1000000; do
ORBHIP_CONE_MAX_WG=$cm timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/c3_bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/c3_bench.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('cone_max $cm C3', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_one_batch_at_a_time_frames_per_s'], e['c3_roofline']['stage_avg_ms'])"
done
