# r06 (late): A/B of the chain kernel (in-tree build against tools/ubench/ab/liborbhip_old.so):
# product-build DAG solve at n = 294 / 342 and the C4 LBA, alternating
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for r in 1 2; do
  for v in new old; do
    if [ $v = old ]; then export ORBHIP_LIB=$PWD/tools/ubench/ab/liborbhip_old.so; else unset ORBHIP_LIB; fi
    echo "== $v"
    timeout -k 10 60 python3 tools/time_dag.py 294 342 2>&1 | grep "n=" || exit 1
    timeout -k 10 60 python3 tools/time_ba.py 50 2>&1 | grep LBA || exit 1
  done
done
