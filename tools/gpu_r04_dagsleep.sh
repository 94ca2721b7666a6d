# r04: the DAG helpers' poll back-off (ORBHIP_DAG_SLEEP, s_sleep units; default 6) against the
# solve time at n = 294 / 570 / 2394 and the C4 LBA
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_dagsleep
mkdir -p $O
for s in 6 1 3 12 6; do
  ORBHIP_DAG_SLEEP=$s timeout -k 10 120 python3 tools/probe_cholesky_dag.py 294:dense 570:dense 2394:loop > $O/p_$s.log 2>&1 || { tail -3 $O/p_$s.log; exit 1; }
  ORBHIP_DAG_SLEEP=$s timeout -k 10 120 python3 tools/time_ba.py 20 > $O/l_$s.log 2>&1 || { tail -3 $O/l_$s.log; exit 1; }
  echo "sleep $s: $(grep -E '^ *(294|570|2394)' $O/p_$s.log | awk '{print $1, $2, $3, $4}' | tr '\n' ' ') | $(grep 'LBA C4' $O/l_$s.log)"
done
