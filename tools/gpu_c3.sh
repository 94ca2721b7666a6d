# C3 check: C3 parity tests (incl. the pipelined batches), then the bench's C3 figures.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_c3_batch_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c3_tests.log 2>&1
rc=$?; tail -3 gpurun_out/c3_tests.log; [ $rc -ne 0 ] && exit $rc
for inf in 2 3; do
timeout -k 10 300 python3 -u bench.py --no-cpu --c3-inflight $inf > gpurun_out/c3_bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/c3_bench.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('C3 inflight', e['c3_batches_in_flight'], e['c3_1280x720_b64_extract_match_frames_per_s'], 'one-at-a-time', e['c3_one_batch_at_a_time_frames_per_s'])"
done
