# Extraction parity (extraction + C3 tests), then the bench's C2 / C3 figures and C3 stage times.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_extract_gpu.py tests/test_c3_batch_gpu.py tests/test_golden.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c3_tests.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
timeout -k 10 300 python3 -u bench.py --no-cpu > gpurun_out/c3_bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/c3_bench.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('C2', d['value'], d['batch1_frames_per_s'], 'C3', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_one_batch_at_a_time_frames_per_s'], e['c3_roofline']['stage_avg_ms'])"
done
