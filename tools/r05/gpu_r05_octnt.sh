# r05: octree threads per level A/B (ORBHIP_OCT_NT 1024 / 512 / 256): extractor tests, device trace, C2 bench
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_octnt
mkdir -p $O
for nt in 512 256; do
  ORBHIP_OCT_NT=$nt timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_frontend.py > $O/pytest_$nt.log 2>&1 || { tail -20 $O/pytest_$nt.log; exit 1; }
  echo "nt=$nt $(tail -1 $O/pytest_$nt.log)"
done
for nt in 1024 512 256; do
  ORBHIP_OCT_NT=$nt ORBHIP_TRACE_BLOCK=0 timeout -k 10 180 python3 -u tools/trace_c2.py > $O/trace_$nt.log 2>&1 || { tail -20 $O/trace_$nt.log; exit 1; }
  echo "nt=$nt"; grep -A2 "k_octree" $O/trace_$nt.log
done
for i in 1 2; do
  for nt in 1024 512 256; do
    ORBHIP_OCT_NT=$nt timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${nt}_$i.json 2> $O/bench_${nt}_$i.err || { tail -5 $O/bench_${nt}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${nt}_$i.json').read().strip().splitlines()[-1]); print('nt=$nt', d['value'], d['batch1_latency_ms'], d['roofline']['stage_avg_ms']['k_octree'])"
  done
done
