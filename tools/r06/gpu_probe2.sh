set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out

timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_nd_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_probe_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_probe_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 600:band 2394:loop > gpurun_out/r06_probe_dag.log 2>&1 || { tail -5 gpurun_out/r06_probe_dag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r06_probe_dag.log | grep -v sub-phases
timeout -k 10 200 python3 -u tools/time_gba.py > gpurun_out/r06_time_gba.log 2>&1 || { tail -5 gpurun_out/r06_time_gba.log; exit 1; }
tail -1 gpurun_out/r06_time_gba.log
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/r06_bench_quick.log 2> gpurun_out/r06_bench_quick.err || { tail -5 gpurun_out/r06_bench_quick.err; exit 1; }
tail -1 gpurun_out/r06_bench_quick.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); e=d['extra']
print('C2', d['value'], 'b1', d['batch1_latency_ms'], 'frac', d['roofline']['frac'], 'C4', e.get('c4_lba_ms'), 'C5', e.get('c5_gba_ms'), 'C3', e.get('c3_1280x720_b64_extract_match_frames_per_s'), 'chol', e.get('c4_roofline'))"
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c4trace -o run -- python3 tools/pmc_workload.py c4lba > gpurun_out/r06_c4trace.log 2>&1 || { tail -5 gpurun_out/r06_c4trace.log; exit 1; }
python3 tools/trace_window.py "$(ls gpurun_out/r06_c4trace/*kernel_trace.csv | head -1)" k_ba_ctl_init 1 > gpurun_out/r06_c4_window.txt 2>&1; cat gpurun_out/r06_c4_window.txt | head -12
