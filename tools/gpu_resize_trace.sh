# Kernel trace of the C3 workload: per-launch k_resize durations by grid (pyramid level).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/rz -o rz -- python3 tools/run_c3.py 4 > gpurun_out/rz.log 2>&1
rc=$?; tail -2 gpurun_out/rz.log; [ $rc -ne 0 ] && exit $rc
f=$(ls gpurun_out/rz/*kernel_trace.csv | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    n = r['Kernel_Name']
    if 'k_resize' in n or 'k_fast_cells' in n or 'k_desc' in n:
        key = (n.split('(')[0], r.get('Grid_Size_X', r.get('Grid_Size', '')), r.get('Grid_Size_Y', ''))
        d[key].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1])):
    v = sorted(v)
    print(k, len(v), 'med %.1f us' % v[len(v) // 2])
PY
