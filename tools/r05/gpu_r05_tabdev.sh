# r05: cone resize tables computed in the kernel (default) against the host's per-tile copies
# (ORBHIP_CONE_TABDEV=0): extractor tests, C2 alternating runs, then the C2 PMC traffic of both
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_tabdev
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_c3_batch_gpu.py tests/test_frontend.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for v in 1 0; do
    ORBHIP_CONE_TABDEV=$v timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail -5 $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('tabdev=$v', d['value'], d['batch1_latency_ms'], r['avg_launch_ms'], r['stage_avg_ms_one_frame_stream']['pyramid (k_pyr_cone | 7x k_resize)'])"
  done
done
for v in 1 0; do
  ORBHIP_CONE_TABDEV=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $O/fetch_$v -o run -- python3 tools/pmc_workload.py c2 > $O/fetch_$v.log 2>&1 || { tail -5 $O/fetch_$v.log; exit 1; }
  ORBHIP_CONE_TABDEV=$v timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $O/write_$v -o run -- python3 tools/pmc_workload.py c2 > $O/write_$v.log 2>&1 || { tail -5 $O/write_$v.log; exit 1; }
  python3 tools/prof_summary.py traffic "$(ls $O/fetch_$v/*counter_collection.csv | head -1)" "$(ls $O/write_$v/*counter_collection.csv | head -1)" $O/traffic_c2_$v.json "c2 tabdev=$v" || exit 1
  python3 -c "import json; d=json.load(open('$O/traffic_c2_$v.json'))['kernels']['k_pyr_cone']; print('tabdev=$v k_pyr_cone', d)"
done
