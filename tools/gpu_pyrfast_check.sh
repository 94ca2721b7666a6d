# k_pyr_fast parity (extraction tests on both paths, stream/frontend parity), trace, C2 A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_extract_gpu.py tests/test_frontend.py tests/test_bench_stream.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/pf_tests.log 2>&1; rc=$?; tail -15 gpurun_out/pf_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/trace_c2.py 2>&1 | grep -v amdgpu.ids
for pf in 1 0; do ORBHIP_PYR_FAST=$pf timeout -k 10 200 python bench.py --no-cpu --no-extra 2>&1 | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('pyr_fast=$pf', d['value'], c['sequential_frames_per_s'], c['host_submit_ms_per_frame'], c['matches_last_pair'], d['roofline']['kernel'], d['roofline']['avg_launch_ms'])"; done
