# r04: C4 LBA kernel trace (which launches a trial makes now), bench C2 section, sharded C5 pieces
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_c4
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_c4/prof -o c4 -- python3 tools/time_ba.py 5 > gpurun_out/r04_c4/prof.log 2>&1 || { tail gpurun_out/r04_c4/prof.log; exit 1; }
grep LBA gpurun_out/r04_c4/prof.log
python3 tools/ba_trace_summary.py "$(ls gpurun_out/r04_c4/prof/*kernel_trace.csv | head -1)" | head -20
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_c4/prof_nd -o nd -- python3 -u tools/time_shard_nd.py 8 > gpurun_out/r04_c4/prof_nd.log 2>&1 || { tail -5 gpurun_out/r04_c4/prof_nd.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_c4/prof_nd.log | tail -3
timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > gpurun_out/r04_c4/bench.log 2> gpurun_out/r04_c4/bench.err || { tail -20 gpurun_out/r04_c4/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_c4/bench.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']
print('value', d['value'], 'batch1', d['batch1_latency_ms'], r['kernel'], r['bound'], r['avg_launch_ms'], r['frac'], r.get('octree_candidates_per_frame'))
print(r['stage_avg_ms'])"
