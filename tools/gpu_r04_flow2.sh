# r04: k_pyr_flow device trace (per-work-group spans, work-group 0's wait / compute cycles per
# task), and the ND back-substitution time in a C5 GBA kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_flow2
mkdir -p $O
ORBHIP_RZ_FLOW=1 timeout -k 10 120 python3 tools/trace_c2.py --c3 > $O/trace_c3_flow.log 2>&1 || { tail -5 $O/trace_c3_flow.log; exit 1; }
grep -v amdgpu.ids $O/trace_c3_flow.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o gba -- python3 -u tools/time_gba.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
grep GBA $O/prof.log
python3 - <<PY
import csv, collections, glob
rows=list(csv.DictReader(open(glob.glob("$O/prof/*kernel_trace.csv")[0])))
agg=collections.defaultdict(list)
for r in rows:
    n=r['Kernel_Name'].replace('orbhip::(anonymous namespace)::','').replace('orbhip::','').split('(')[0]
    agg[n].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k,v in sorted(agg.items(), key=lambda x:-sum(x[1]))[:8]: print(k, len(v), round(sum(v)/len(v),2))
PY
