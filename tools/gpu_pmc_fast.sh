# One SQ pass (instruction mix, stall split) over the C3 workload: where k_fast_cells / k_desc / k_resize spend issue.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcf
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE"
for pass in p1 p2; do
  case $pass in p1) ctr="$P1";; p2) ctr="$P2";; esac
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/pmcf/$pass -o run \
      -- python3 tools/pmc_workload.py c3 > gpurun_out/pmcf/$pass.log 2>&1
  rc=$?; echo "$pass rc=$rc"; [ $rc -ne 0 ] && { tail -5 gpurun_out/pmcf/$pass.log; exit $rc; }
done
python3 - <<'PY'
import csv, glob, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob('gpurun_out/pmcf/*/*counter_collection.csv'):
    for r in csv.DictReader(open(f)):
        n = r['Kernel_Name'].split('(')[0].replace('void ', '')
        agg[n][r['Counter_Name']].append(float(r['Counter_Value']))
for n, d in agg.items():
    if not any(k in n for k in ('fast', 'desc', 'resize', 'octree', 'match')): continue
    print(n, {k: round(sum(v) / max(1, len(v) // 1), 1) for k, v in sorted(d.items())})
PY
