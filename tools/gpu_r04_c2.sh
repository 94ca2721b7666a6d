# r04: C2 front-end checks (parity tests of the front-end and the cone) and two C2 bench lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_c2
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_frontend.py tests/test_extract_gpu.py tests/test_bench_stream.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra > $O/b_$i.log 2> $O/b_$i.err || { tail -5 $O/b_$i.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/b_$i.log') if l.startswith('{')][-1]); r=d['roofline']
print('value', d['value'], 'batch1', d['batch1_latency_ms'], r['kernel'], r['avg_launch_ms'], r['frac'], r['stage_avg_ms'])"
done
