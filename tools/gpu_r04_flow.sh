# r04: one-launch dataflow pyramid (ORBHIP_RZ_FLOW=1): parity tests, kernel trace of the C3 batch
# workload and the bench's C3 lines with it on
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_flow}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_c3_batch_gpu.py tests/test_extract_gpu.py -k "flow or c3_batch_vs" -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
ORBHIP_RZ_FLOW=1 timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o c3 -- python3 tools/pmc_workload.py c3 > $O/c3prof.log 2>&1 || { tail -5 $O/c3prof.log; exit 1; }
python3 tools/prof_summary.py stats "$(ls $O/c3prof/*kernel_stats.csv | head -1)" $O/c3_kernel_stats.md "ORBHIP_RZ_FLOW=1 tools/pmc_workload.py c3" || exit 1
head -14 $O/c3_kernel_stats.md | tail -8
ORBHIP_RZ_FLOW=1 timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -v amdgpu.ids $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); e=d['extra']
print('c3', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_one_batch_at_a_time_frames_per_s'], e['c3_roofline']['stage_avg_ms'], e['c3_hbm_stage'])"
