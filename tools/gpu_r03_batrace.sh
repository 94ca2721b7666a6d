# r03: kernel traces of single C4 LBA solves and one C5 GBA (per-kernel durations and gaps).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_lba -o lba -- python3 tools/time_ba.py 5 0 > gpurun_out/tr_lba.log 2>&1 || { tail gpurun_out/tr_lba.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_gba -o gba -- python3 tools/time_gba.py 400 20000 10 > gpurun_out/tr_gba.log 2>&1 || { tail gpurun_out/tr_gba.log; exit 1; }
grep -v amdgpu.ids gpurun_out/tr_lba.log gpurun_out/tr_gba.log
find gpurun_out/tr_lba gpurun_out/tr_gba -name '*kernel_trace.csv'
