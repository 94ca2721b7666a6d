# r06: one-GPU GBA time against the problem size (the sharded-C5 crossover model)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for sz in "400 20000" "400 80000" "400 200000" "1000 50000" "2000 100000"; do
  timeout -k 10 120 python3 -u tools/time_gba.py $sz 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/r06_gba_sizes.log || exit 1
done
