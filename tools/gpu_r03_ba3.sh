# r03: BA parity tests, LBA / GBA timing, host-side phase split of one LBA (ORBHIP_BA_TIMING)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_sharded_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_ba.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_ba.log; [ $rc -eq 0 ] || exit $rc
timeout -k 5 120 python3 -u tools/time_ba.py 20 0 2>&1 | grep -v amdgpu.ids || exit 1
ORBHIP_BA_TIMING=1 timeout -k 5 120 python3 -u tools/time_ba.py 3 0 2>&1 | grep -v amdgpu.ids | tail -3 || exit 1
timeout -k 5 120 python3 -u tools/time_gba.py 400 20000 10 2>&1 | grep -v amdgpu.ids
