# r03: the default bench line, then a rocprofv3 kernel trace of the bench's C2 section alone
# (bench.py --no-extra --no-cpu: the launches the headline roofline's live timing covers).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_sel.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 500 python3 -u bench.py > gpurun_out/r03_bench.log 2> gpurun_out/r03_bench.err || { tail -20 gpurun_out/r03_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/r03_bench.log | tail -1 > gpurun_out/r03_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_c2prof -o c2 \
    -- python3 -u bench.py --no-extra --no-cpu > gpurun_out/r03_c2prof.log 2>&1 || { tail -20 gpurun_out/r03_c2prof.log; exit 1; }
python3 tools/prof_summary.py stats "$(ls gpurun_out/r03_c2prof/*kernel_stats.csv | head -1)" \
    gpurun_out/r03_c2_kernel_stats.md "bench.py --no-extra --no-cpu (the C2 section)" || exit 1
head -12 gpurun_out/r03_c2_kernel_stats.md
python3 -c "
import json; d=json.load(open('gpurun_out/r03_bench.json')); r=d['roofline']
print('value', d['value'], 'batch1', d['batch1_latency_ms'], r['kernel'], r['avg_launch_ms'], r['frac'], r['stage_avg_ms'])
e=d.get('extra',{}); print({k: (v.get('kernel'), v.get('avg_launch_ms'), v.get('frac'), v.get('bound')) for k,v in e.items() if 'roofline' in k})
print({k: v for k,v in e.items() if not isinstance(v, dict)})
print(d.get('cpu_baseline'))"
