# r05: FAST pair-window pitch 63 (main) against r04's 48 (pwp48): extractor tests, C3 and C2 alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_pwp
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_c3_batch_gpu.py tests/test_frontend.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in main pwp48; do
    unset ORBHIP_LIB
    [ $v = main ] || export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so
    echo "$v $(timeout -k 10 300 python3 -u tools/time_c3.py 10 2>/dev/null | tail -1)" || exit 1
    timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail -5 $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v C2', d['value'], d['batch1_latency_ms'], r['stage_avg_ms_one_frame_stream']['k_fast_cells'])"
  done
done
