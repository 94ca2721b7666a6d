# r02 baseline: default bench line + rocprofv3 kernel stats of the same command without the CPU leg.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu > gpurun_out/prof.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/bench.log | tail -c 4000; exit $rc
