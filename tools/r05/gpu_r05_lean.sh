# r05: C3 A/B of the lean pair-test round (main) against r04's form (lean0), alternating runs; the
# C2 section with the cone's per-tile tables (default) and the compact ones; extractor tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_lean
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_c3_batch_gpu.py tests/test_frontend.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  for v in main lean0; do
    if [ $v = main ]; then unset ORBHIP_LIB; else export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so; fi
    timeout -k 10 300 python3 -u tools/time_c3.py 10 2>/dev/null | tail -1 || exit 1
  done
done
unset ORBHIP_LIB
for v in tile level tile level; do
  ORBHIP_CONE_TABS=$v timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['batch1_latency_ms'], d['roofline']['avg_launch_ms'])"
done
