set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_init -o run -- python3 tools/time_init.py > gpurun_out/prof_init.log 2>&1; rc=$?
cut -d, -f1-8 gpurun_out/prof_init/run_kernel_stats.csv | head -20; exit $rc
