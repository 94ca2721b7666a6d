# SQ counters of the C3 kernels (one pass, kernel-trace only): VALU / LDS issue, wave cycles and stalls.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_c3 -o c3 -- python3 tools/run_c3.py 3 > gpurun_out/pmc_c3.log 2>&1
rc=$?; tail -2 gpurun_out/pmc_c3.log; exit $rc
