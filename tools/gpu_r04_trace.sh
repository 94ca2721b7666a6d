# r04: device phase trace of one C3 batch and one C2 step, then the C3 PMC passes (counters and
# HBM traffic per kernel)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_trace
timeout -k 10 120 python3 tools/trace_c2.py --c3 > gpurun_out/r04_trace/c3.log 2>&1 || { tail -5 gpurun_out/r04_trace/c3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_trace/c3.log
timeout -k 10 120 python3 tools/trace_c2.py > gpurun_out/r04_trace/c2.log 2>&1 || { tail -5 gpurun_out/r04_trace/c2.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r04_trace/c2.log
REGIMES="${REGIMES:-c3}" PFX=r04 bash tools/gpu_pmc.sh || exit 1
python3 -c "
import json
t=json.load(open('gpurun_out/pmc/traffic_c3.json'))
for k,v in t['kernels'].items(): print(k, v)
c=json.load(open('gpurun_out/pmc/counters.json'))
for r,kk in c.items():
    if not isinstance(kk, dict): continue
    for k,v in kk.items():
        if isinstance(v, dict): print(r, k, {a: v.get(a) for a in ('duration_us','valu_issue_frac','lds_issue_frac','wave_time_split')})
"
