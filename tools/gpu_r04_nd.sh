# r04: nested dissection — parity tests, solve timing per segment count, C5 GBA time
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_nd
timeout -k 10 300 python3 -u -m pytest tests/test_nd_gpu.py -m gpu -v -x --timeout 120 --timeout-method thread > gpurun_out/r04_nd/pytest.log 2>&1
rc=$?; grep -E "passed|failed|PASS|FAIL" gpurun_out/r04_nd/pytest.log | tail -20; [ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/r04_nd/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 -u tools/probe_nd.py > gpurun_out/r04_nd/probe.log 2>&1 || { tail -5 gpurun_out/r04_nd/probe.log; exit 1; }
cat gpurun_out/r04_nd/probe.log
timeout -k 10 120 python3 -u tools/time_gba.py > gpurun_out/r04_nd/gba.log 2>&1 || exit 1
cat gpurun_out/r04_nd/gba.log
ORBHIP_ND=0 timeout -k 10 120 python3 -u tools/time_gba.py > gpurun_out/r04_nd/gba_plain.log 2>&1 || exit 1
cat gpurun_out/r04_nd/gba_plain.log
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_concurrent_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > gpurun_out/r04_nd/pytest_ba.log 2>&1
rc=$?; tail -3 gpurun_out/r04_nd/pytest_ba.log; exit $rc
