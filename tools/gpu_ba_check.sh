set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python tools/probe_cholesky_reg.py 294 > gpurun_out/probe_reg.log 2>&1; rc=$?; cat gpurun_out/probe_reg.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py -x -q > gpurun_out/ba_tests.log 2>&1; rc=$?; tail -5 gpurun_out/ba_tests.log; [ $rc -le 1 ] || exit $rc
ORBHIP_BA_TIMING=1 timeout -k 10 200 python tools/time_ba.py 20 128 && ORBHIP_BA_TIMING=1 timeout -k 10 200 python tools/time_ba.py 2 256 > gpurun_out/time_ba.log 2>&1; rc=$?; tail -8 gpurun_out/time_ba.log; exit $rc
