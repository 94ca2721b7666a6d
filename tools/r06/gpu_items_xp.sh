# r06: k_ba_schur_items cost split (tree / barrier) on A/B builds, C4 trace windows
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in base notree nobar base; do
  ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_xp_$v -o run -- python3 tools/pmc_workload.py c4lba > gpurun_out/r06_xp_$v.log 2>&1 || exit 1
  echo "== $v"; python3 tools/trace_window.py "$(ls gpurun_out/r06_xp_$v/*kernel_trace.csv | head -1)" k_ba_ctl_init 1 2>&1 | grep -E "window|schur_items|backsub|k_ba_lin"
done
