# r04: C4 trace after the LDS-pose fused kernel, host timing split, BA tests; the bench C2 section
# under rocprofv3 (its own device-stamped avg_launch_ms vs the trace of the same launches)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_c4b
timeout -k 10 300 python3 -u -m pytest tests/test_ba_sharded_nd_gpu.py tests/test_ba_gpu.py tests/test_ba_concurrent_gpu.py tests/test_nd_gpu.py tests/test_ba_sharded_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r04_c4b/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r04_c4b/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04_c4b/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 tools/time_ba.py 20 > gpurun_out/r04_c4b/lba.log 2>&1 || exit 1
grep LBA gpurun_out/r04_c4b/lba.log
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 tools/time_ba.py 3 > gpurun_out/r04_c4b/lba_timing.log 2>&1 || exit 1
grep "timing B=1" gpurun_out/r04_c4b/lba_timing.log | tail -2
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_c4b/prof -o c4 -- python3 tools/time_ba.py 5 > gpurun_out/r04_c4b/prof.log 2>&1 || { tail gpurun_out/r04_c4b/prof.log; exit 1; }
python3 tools/ba_trace_summary.py "$(ls gpurun_out/r04_c4b/prof/*kernel_trace.csv | head -1)" | head -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_c4b/c2prof -o c2 -- python3 -u bench.py --no-extra --no-cpu > gpurun_out/r04_c4b/c2prof.log 2>&1 || { tail -20 gpurun_out/r04_c4b/c2prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_c4b/c2prof.log | grep '"metric"' | tail -1 > gpurun_out/r04_c4b/c2prof_bench.json
python3 tools/prof_summary.py sections "$(ls gpurun_out/r04_c4b/c2prof/*kernel_trace.csv | head -1)" gpurun_out/r04_c4b/c2_sections.md 20 200 || exit 1
tail -12 gpurun_out/r04_c4b/c2_sections.md
python3 -c "
import json; d=json.load(open('gpurun_out/r04_c4b/c2prof_bench.json')); r=d['roofline']
print('profiled bench: value', d['value'], r['kernel'], r['avg_launch_ms'], r['stage_avg_ms'])"
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_c4b/prof_nd -o nd -- python3 -u tools/time_shard_nd.py 8 > gpurun_out/r04_c4b/prof_nd.log 2>&1 || { tail -5 gpurun_out/r04_c4b/prof_nd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_c4b/prof_nd.log | grep "ms " | tail -3
timeout -k 10 120 python3 -u tools/time_gba.py > gpurun_out/r04_c4b/gba.log 2>&1 && grep GBA gpurun_out/r04_c4b/gba.log
