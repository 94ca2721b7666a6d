# r06 A/B: FAST pair-window pitch 68 (= dc 36 mod 32: each half-wave of the pair test reads consecutive banks) vs 48
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2 3; do
for v in p48 p68; do
  ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so timeout -k 10 120 python3 tools/time_c3.py 10 2>&1 | grep -v amdgpu.ids | tail -1
done
done
ORBHIP_LIB=tools/ubench/ab/liborbhip_p68.so timeout -k 10 300 python3 -u -m pytest tests/test_c3_batch_gpu.py tests/test_extract_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -2
