# Kernel trace of single C4 LBA solves (no batch): per-solve kernel time vs wall time.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_lba1 -o lba -- python3 tools/time_ba.py 5 0 > gpurun_out/prof_lba1.log 2>&1
rc=$?; cat gpurun_out/prof_lba1.log | grep -v amdgpu.ids; exit $rc
