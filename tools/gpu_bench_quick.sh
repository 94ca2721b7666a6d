# Quick validation of bench.py on the box (+ the counter list for the PMC passes).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || echo "rocprofv3 -L rc=$?"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench_quick.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/bench_quick.log | tail -c 6000; exit $rc
