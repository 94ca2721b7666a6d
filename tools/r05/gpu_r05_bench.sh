# r05: default bench run (one JSON line) on one MI355X
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_bench}
mkdir -p $O
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.err; rc=$?
tail -c 6000 $O/bench.json; tail -5 $O/bench.err
exit $rc
