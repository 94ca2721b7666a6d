# r04: extractor change check: the extraction parity tests, then the C2 / C3 bench lines and a
# kernel trace of the C3 batch workload (k_fast_cells per-launch time)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_fast}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_extract_gpu.py tests/test_c3_batch_gpu.py tests/test_frontend.py tests/test_match_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c3prof -o c3 -- python3 tools/pmc_workload.py c3 > $O/c3prof.log 2>&1 || { tail -5 $O/c3prof.log; exit 1; }
python3 tools/prof_summary.py stats "$(ls $O/c3prof/*kernel_stats.csv | head -1)" $O/c3_kernel_stats.md "tools/pmc_workload.py c3" || exit 1
head -14 $O/c3_kernel_stats.md | tail -8
timeout -k 10 400 python3 -u bench.py --no-cpu > $O/bench.log 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
grep -v amdgpu.ids $O/bench.log | tail -1 > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); r=d['roofline']; e=d['extra']
print('value', d['value'], 'batch1', d['batch1_latency_ms'], r['stage_avg_ms'])
print('c3', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_roofline']['stage_avg_ms'])"
