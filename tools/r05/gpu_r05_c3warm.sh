# r05: is the c3 k_fast_cells trace duration a warm-up effect? 16 vs 96 batches, plain kernel trace
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for n in 96 16; do
  PMC_C3_STEPS=$n timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/c3w${n} -o run \
      -- python3 tools/pmc_workload.py c3 > gpurun_out/pmc/c3w${n}.log 2>&1 || { tail -5 gpurun_out/pmc/c3w${n}.log; exit 1; }
  python3 tools/prof_summary.py stats "$(ls gpurun_out/pmc/c3w${n}/*kernel_stats.csv | head -1)" \
      gpurun_out/pmc/r05_c3w${n}_kernel_stats.md "PMC_C3_STEPS=$n tools/pmc_workload.py c3" || exit 1
  grep k_fast_cells gpurun_out/pmc/r05_c3w${n}_kernel_stats.md
  python3 - <<PY
import csv,glob
f=glob.glob('gpurun_out/pmc/c3w${n}/*kernel_trace.csv')[0]
d=[(int(r['Start_Timestamp']),int(r['End_Timestamp'])) for r in csv.DictReader(open(f)) if r['Kernel_Name'].startswith('k_fast_cells')]
d.sort(); us=[(e-s)/1000 for s,e in d]
print('n=${n} first8', [round(x) for x in us[:8]], 'last8', [round(x) for x in us[-8:]])
PY
done
