# r03: DAG Cholesky phase timings vs helper count and helper poll back-off
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for cfg in "0 6" "0 2" "0 30" "0 100" "16 6" "64 6"; do
  set -- $cfg
  echo "helpers=$1 sleep=$2"
  ORBHIP_DAG_HELPERS=$1 ORBHIP_DAG_SLEEP=$2 timeout -k 5 60 python3 -u tools/probe_cholesky_dag.py 294:dense 2394:loop 2>&1 | grep -v amdgpu.ids || exit 1
done
