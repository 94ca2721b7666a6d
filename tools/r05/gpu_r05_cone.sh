# r05: C2 device trace (cone / octree phases) and the C2 bench section, extractor parity tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_oct5
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_frontend.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
ORBHIP_TRACE_BLOCK=0 timeout -k 10 180 python3 -u tools/trace_c2.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -v amdgpu.ids $O/trace.log
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_$i.json 2> $O/bench_$i.err || { tail -5 $O/bench_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]); print('bench', d['value'], d['batch1_latency_ms'], d['roofline']['avg_launch_ms'], d['roofline']['stage_avg_ms'])"
done
