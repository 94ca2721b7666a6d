set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ba -o ba -- python3 tools/time_ba.py 5 128 > gpurun_out/prof_ba.log 2>&1
echo rc=$?
