# r04: sharded BA by segments (device-driven, collectives on the stream) + the BA suites
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_shard
timeout -k 10 600 python3 -u -m pytest tests/test_ba_sharded_nd_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_gpu.py tests/test_nd_gpu.py tests/test_ba_concurrent_gpu.py -m gpu -v -x --timeout 200 --timeout-method thread > gpurun_out/r04_shard/pytest.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/r04_shard/pytest.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" gpurun_out/r04_shard/pytest.log | head -30; exit $rc; }
timeout -k 10 120 python3 -u tools/time_gba.py > gpurun_out/r04_shard/gba.log 2>&1 || exit 1
cat gpurun_out/r04_shard/gba.log
timeout -k 10 120 python3 -u tools/time_ba.py 20 > gpurun_out/r04_shard/lba.log 2>&1 || exit 1
cat gpurun_out/r04_shard/lba.log
(cd tools/ubench && timeout -k 5 60 ./ubench_f64 > ../../gpurun_out/r04_shard/ubench_f64.log 2>&1 && timeout -k 5 60 ./diag16 > ../../gpurun_out/r04_shard/diag16.log 2>&1) || exit 1
cat gpurun_out/r04_shard/ubench_f64.log gpurun_out/r04_shard/diag16.log | grep -v amdgpu.ids
timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/r04_shard/bench.log 2> gpurun_out/r04_shard/bench.err || { tail -20 gpurun_out/r04_shard/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_shard/bench.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('value', d['value'], 'batch1', d['batch1_latency_ms'], r['kernel'], r['bound'], r['avg_launch_ms'], r['frac'], r.get('octree_candidates_per_frame'))
print(r['stage_avg_ms'])"
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_shard/prof_nd -o nd -- python3 -u tools/time_shard_nd.py 8 > gpurun_out/r04_shard/prof_nd.log 2>&1 || { tail -5 gpurun_out/r04_shard/prof_nd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_shard/prof_nd.log | tail -3
