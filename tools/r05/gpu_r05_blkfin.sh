# r05: octree FINAL passes by the whole block (main) against wave 0 (noblk): C2 section alternating runs,
# then one device trace of main
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_blkfin
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_frontend.py tests/test_match_gpu.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in main noblk; do
    unset ORBHIP_LIB
    [ $v = main ] || export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so
    timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail -5 $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', d['value'], d['batch1_latency_ms'], r['avg_launch_ms'], r['stage_avg_ms_one_frame_stream'])"
  done
done
unset ORBHIP_LIB
ORBHIP_TRACE_BLOCK=0 timeout -k 10 180 python3 -u tools/trace_c2.py > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -v "per-wg\|amdgpu.ids" $O/trace.log
