# r06 A/B on one box: waves 2/3 prefetching the next interval's inputs (pf) against the plain form (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for i in 1 2; do
for v in pro0 pro1; do
  echo "== $v"
  ORBHIP_PROBE_LIB=tools/ubench/ab/liborbhip_$v.so timeout -k 10 60 python3 -u tools/probe_cholesky_dag.py 294:dense 2394:loop 2>&1 | grep -v amdgpu.ids | grep "n=" | cut -c1-200
done
done
