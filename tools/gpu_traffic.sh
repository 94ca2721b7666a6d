# FETCH_SIZE / WRITE_SIZE passes only (HBM bytes per launch) for the given regimes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
for regime in ${REGIMES:-c2 c3}; do
  for pass in fetch write; do
    case $pass in fetch) ctr="FETCH_SIZE";; write) ctr="WRITE_SIZE";; esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/pmc/${regime}_${pass} -o run \
        -- python3 tools/pmc_workload.py $regime > gpurun_out/pmc/${regime}_${pass}.log 2>&1
    rc=$?; echo "$regime $pass rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${regime}_${pass}.log; exit $rc; fi
  done
  f() { ls gpurun_out/pmc/${regime}_$1/*counter_collection.csv | head -1; }
  python3 tools/prof_summary.py traffic "$(f fetch)" "$(f write)" gpurun_out/pmc/traffic_${regime}.json "$regime" || exit 1
done
