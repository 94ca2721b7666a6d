# r05: k_fast_cells threads per cell (ORBHIP_FAST_NT) on the 16-camera C2 stream, alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_fastnt
mkdir -p $O
for i in 1 2; do
  for t in 256 512 1024; do
    ORBHIP_FAST_NT=$t timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${t}_$i.json 2> $O/bench_${t}_$i.err || { tail -5 $O/bench_${t}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${t}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('fastnt=$t', d['value'], d['batch1_latency_ms'], r['avg_launch_ms'], r.get('stage_avg_ms'))"
  done
done
