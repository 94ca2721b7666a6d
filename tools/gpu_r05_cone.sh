# r05: FETCH/WRITE_SIZE calibration for 4-B reads and 1-B stores; k_pyr_cone traffic with the
# compact per-level tables vs the per-tile copies, and with XCD-grouped tiles; extractor tests; C2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_cone
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/cal_$c -o cal -- ./tools/ubench/fetch_cal > $O/cal_$c.log 2>&1 || { tail -5 $O/cal_$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    f = glob.glob(f"gpurun_out/r05_cone/cal_{c}/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] == c:
            acc[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
    print(c, {k: [round(x / 1024, 1) for x in v] for k, v in acc.items()}, "(MiB per launch)")
PY
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_frontend.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in compact tile grouped; do
  case $v in compact) env="";; tile) env="ORBHIP_CONE_TABS=tile";; grouped) env="ORBHIP_XCD_RUN=8";; esac
  for c in FETCH_SIZE WRITE_SIZE; do
    if [ -n "$env" ]; then export ${env%%=*}=${env#*=}; fi
    timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/${v}_$c -o run -- python3 tools/pmc_workload.py c2 > $O/${v}_$c.log 2>&1 || { tail -5 $O/${v}_$c.log; exit 1; }
    unset ORBHIP_CONE_TABS ORBHIP_XCD_RUN
  done
  python3 tools/prof_summary.py traffic "$(ls $O/${v}_FETCH_SIZE/*counter_collection.csv | head -1)" "$(ls $O/${v}_WRITE_SIZE/*counter_collection.csv | head -1)" $O/traffic_$v.json c2 || exit 1
  python3 -c "import json; d=json.load(open('$O/traffic_$v.json'))['kernels']; print('$v', {k: (v['fetch_kb_raw'], v['write_kb'], v['hbm_bytes_per_launch']) for k, v in d.items() if k in ('k_pyr_cone', 'k_fast_cells', 'k_desc_kp')})"
done
for v in compact grouped; do
  if [ $v = grouped ]; then export ORBHIP_XCD_RUN=8; fi
  timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_$v.json 2> $O/bench_$v.err || { tail -5 $O/bench_$v.err; exit 1; }
  unset ORBHIP_XCD_RUN
  python3 -c "import json; d=json.loads(open('$O/bench_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['batch1_latency_ms'], d['roofline']['avg_launch_ms'])"
done
