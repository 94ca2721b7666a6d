# final tree of a round (R=r06 default): the whole -m gpu suite, smoke, the default bench line, and a rocprofv3 kernel
# trace of the bench's C2 section (the headline roofline's reproduction); logs under gpurun_out/
# for profiles/. Stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
R=${R:-r06}
mkdir -p gpurun_out
echo "[1/4] pytest -m gpu"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/${R}_pytest_gpu.log 2>&1
rc=$?; grep -E "passed|failed" gpurun_out/${R}_pytest_gpu.log | tail -3; [ $rc -eq 0 ] || { grep -E "FAILED|ERROR" gpurun_out/${R}_pytest_gpu.log | head; exit $rc; }
echo "[2/4] smoke"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1 || { tail -5 gpurun_out/${R}_smoke.log; exit 1; }
tail -1 gpurun_out/${R}_smoke.log
echo "[3/4] bench"
timeout -k 10 600 python3 -u bench.py > gpurun_out/${R}_bench.log 2> gpurun_out/${R}_bench.err || { tail -20 gpurun_out/${R}_bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/${R}_bench.log | tail -1 > gpurun_out/${R}_bench.json
echo "[4/4] rocprofv3 of the C2 section"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_c2prof -o c2 \
    -- python3 -u bench.py --no-extra --no-cpu > gpurun_out/${R}_c2prof.log 2>&1 || { tail -20 gpurun_out/${R}_c2prof.log; exit 1; }
python3 tools/prof_summary.py stats "$(ls gpurun_out/${R}_c2prof/*kernel_stats.csv | head -1)" \
    gpurun_out/${R}_c2_kernel_stats.md "bench.py --no-extra --no-cpu (the C2 section)" || exit 1
python3 tools/prof_summary.py sections "$(ls gpurun_out/${R}_c2prof/*kernel_trace.csv | head -1)" \
    gpurun_out/${R}_c2_kernel_stats.md 20 200 || exit 1
grep -v amdgpu.ids gpurun_out/${R}_c2prof.log | tail -1 > gpurun_out/${R}_c2prof_bench.json
head -10 gpurun_out/${R}_c2_kernel_stats.md
python3 -c "
import json; d=json.load(open('gpurun_out/'+'${R}'+'_bench.json')); r=d['roofline']
print('value', d['value'], 'batch1', d['batch1_latency_ms'], r['kernel'], r['avg_launch_ms'], r['frac'])
e=d.get('extra',{}); print({k: (v.get('kernel'), v.get('avg_launch_ms'), v.get('frac'), v.get('bound')) for k,v in e.items() if 'roofline' in k or 'hbm' in k})
print({k: v for k,v in e.items() if not isinstance(v, dict)})
print(d.get('cpu_baseline'))"
