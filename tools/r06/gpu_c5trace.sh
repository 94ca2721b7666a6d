# r06: C5 GBA kernel trace (last solve of tools/time_gba.py) and the C4 host split
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c5trace -o run -- python3 tools/time_gba.py > gpurun_out/r06_c5trace.log 2>&1 || { tail -5 gpurun_out/r06_c5trace.log; exit 1; }
python3 tools/trace_window.py "$(ls gpurun_out/r06_c5trace/*kernel_trace.csv | head -1)" k_ba_ctl_init 1 2>&1 | head -16
ORBHIP_BA_TIMING=1 timeout -k 10 60 python3 tools/time_ba.py 20 2>&1 | grep -v amdgpu.ids | tail -3
