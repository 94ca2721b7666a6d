# The default bench line alone (reads the committed profiles/ counters and traffic).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.log | tail -1 | cut -c1-300
