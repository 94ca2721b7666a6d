set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in ${KS:-2 3 4}; do
timeout -k 10 300 python3 -u bench.py --no-cpu --steps 50 --c3-inflight $k > gpurun_out/infl.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/infl.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('inflight=$k', 'C3', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_one_batch_at_a_time_frames_per_s'])"
done
