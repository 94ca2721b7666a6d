# r05: plain rocprofv3 kernel traces (no counters) of the c3 and c4 workloads on the final tree,
# the durations the bench's live c3_roofline / c4_roofline timings are checked against
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for regime in c3 c4; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/${regime}_stats -o run \
      -- python3 tools/pmc_workload.py $regime > gpurun_out/pmc/${regime}_stats.log 2>&1
  rc=$?; echo "$regime stats rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${regime}_stats.log; exit $rc; fi
  python3 tools/prof_summary.py stats "$(ls gpurun_out/pmc/${regime}_stats/*kernel_stats.csv | head -1)" \
      gpurun_out/pmc/r05_${regime}_kernel_stats.md "tools/pmc_workload.py $regime" || exit 1
  head -12 gpurun_out/pmc/r05_${regime}_kernel_stats.md
done
