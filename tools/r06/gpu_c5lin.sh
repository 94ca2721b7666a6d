set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in 1 4 1 4; do
  ORBHIP_LIN_PPW=$v timeout -s KILL 150 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c5lin$v -o run -- python3 tools/time_gba.py > gpurun_out/r06_c5lin$v.log 2>&1 || { tail -5 gpurun_out/r06_c5lin$v.log; exit 1; }
  echo "PPW=$v $(grep GBA gpurun_out/r06_c5lin$v.log) | $(grep -h '"k_ba_lin' gpurun_out/r06_c5lin$v/*kernel_stats.csv | cut -d, -f1-5)"
done
