# r05: timing probe of the trial's agent-scope (sc1) error / point stores in the fused LBA trial:
# main against plain stores (plainerr, unsafe beside the controller's refresh), alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for i in 1 2 3; do
  for v in main plainerr; do
    unset ORBHIP_LIB
    [ $v = main ] || export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so
    echo "$v $(timeout -k 10 120 python3 -u tools/time_ba.py 40 2>/dev/null | tail -1)" || exit 1
  done
done
