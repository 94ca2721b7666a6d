# C2 host-submission experiment (cameras x host threads) + kernel trace of single C4 LBA solves.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 240 python3 -u tools/multi_thread_c2.py 300 > gpurun_out/multi_thread_c2.log 2>&1
rc=$?; cat gpurun_out/multi_thread_c2.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/prof_lba1 -o lba -- python3 tools/time_ba.py 5 0 > gpurun_out/prof_lba1.log 2>&1
rc=$?; cat gpurun_out/prof_lba1.log | grep -v amdgpu.ids; exit $rc
