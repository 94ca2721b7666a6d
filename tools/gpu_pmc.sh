# rocprofv3 PMC passes per regime (MI355X_MICROARCH.md: one pass per counter group, kernel-trace
# only, FETCH_SIZE and WRITE_SIZE in passes of their own), then the committed summaries:
#   profiles/traffic_<regime>.json   HBM bytes per launch (FETCH x2 + WRITE)
#   profiles/counters.json           VALU / LDS / MFMA activity per launch
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
for regime in ${REGIMES:-c2 c3 c4 c5}; do
  # plain kernel trace of the same workload (the durations the bench's live timing is checked against)
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc/${regime}_stats -o run \
      -- python3 tools/pmc_workload.py $regime > gpurun_out/pmc/${regime}_stats.log 2>&1
  rc=$?; echo "$regime stats rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${regime}_stats.log; exit $rc; fi
  python3 tools/prof_summary.py stats "$(ls gpurun_out/pmc/${regime}_stats/*kernel_stats.csv | head -1)" \
      gpurun_out/pmc/${PFX:-r03}_${regime}_kernel_stats.md "tools/pmc_workload.py $regime" || exit 1
  for pass in p1 p2 fetch write; do
    case $pass in
      p1) ctr="$P1";; p2) ctr="$P2";; fetch) ctr="FETCH_SIZE";; write) ctr="WRITE_SIZE";;
    esac
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d gpurun_out/pmc/${regime}_${pass} -o run \
        -- python3 tools/pmc_workload.py $regime > gpurun_out/pmc/${regime}_${pass}.log 2>&1
    rc=$?; echo "$regime $pass rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 gpurun_out/pmc/${regime}_${pass}.log; exit $rc; fi
  done
  f() { ls gpurun_out/pmc/${regime}_$1/*counter_collection.csv | head -1; }
  python3 tools/prof_summary.py traffic "$(f fetch)" "$(f write)" gpurun_out/pmc/traffic_${regime}.json "$regime" || exit 1
done
python3 tools/prof_summary.py counters gpurun_out/pmc gpurun_out/pmc/counters.json ${REGIMES:-c2 c3 c4 c5}
