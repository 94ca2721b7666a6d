# r06: k_fast_cells with 32 lanes per window row (bank-conflict-free pair test): extract / C3 parity,
# then the C3 kernel trace and its LDS conflict counters
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_extract_gpu.py tests/test_c3_batch_gpu.py tests/test_golden.py tests/test_frontend.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_fast_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_fast_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c3stats -o run -- python3 tools/pmc_workload.py c3 > gpurun_out/r06_c3stats.log 2>&1 || { tail -5 gpurun_out/r06_c3stats.log; exit 1; }
python3 tools/prof_summary.py stats "$(ls gpurun_out/r06_c3stats/*kernel_stats.csv | head -1)" gpurun_out/r06_c3_kernel_stats.md "tools/pmc_workload.py c3" && head -12 gpurun_out/r06_c3_kernel_stats.md
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/r06_c3pmc -o run -- python3 tools/pmc_workload.py c3 > gpurun_out/r06_c3pmc.log 2>&1 || { tail -5 gpurun_out/r06_c3pmc.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob('gpurun_out/r06_c3pmc/*counter_collection.csv')[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open(f)):
    if 'k_fast_cells' not in r['Kernel_Name']: continue
    acc['k_fast_cells'][r['Counter_Name']] += float(r['Counter_Value'])
    n[(r['Counter_Name'])] += 1
for k, d in acc.items():
    print(k, {c: v / max(1, n[c]) for c, v in d.items()})
PY
