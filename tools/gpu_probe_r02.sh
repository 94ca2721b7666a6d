# Host CPU probe + C4 timing breakdown (single and B=256) + kernel stats of the batched solve.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
{ nproc; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())";
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E "Model name|Socket|Core|Thread|NUMA node\(s\)|^CPU\(s\)"; 
  echo OMP=$OMP_NUM_THREADS; free -g | head -2; } > gpurun_out/host_probe.txt 2>&1
cat gpurun_out/host_probe.txt
ORBHIP_BA_TIMING=1 timeout -k 10 200 python3 tools/time_ba.py 10 256 > gpurun_out/time_ba.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/time_ba.log | tail -8; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lbab -o lba -- python3 tools/time_ba.py 2 256 > gpurun_out/prof_lbab.log 2>&1
rc=$?; f=$(ls gpurun_out/prof_lbab/*kernel_stats.csv | head -1); python3 tools/prof_summary.py stats "$f" gpurun_out/lbab_stats.md "C4 batched"; head -30 gpurun_out/lbab_stats.md; exit $rc
