# r04: batch match chunk size (ORBHIP_MATCH_TC 256 / 512 / 1024): parity at 1024 and 512, then per
# setting the C3 batch workload's kernel trace and FETCH_SIZE / WRITE_SIZE passes for k_match_top2
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_match
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_extract_gpu.py tests/test_frontend.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_extract.log 2>&1
rc=$?; tail -1 $O/pytest_extract.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_extract.log | head -20; exit $rc; }
for tc in 1024 512; do
  ORBHIP_MATCH_TC=$tc timeout -k 10 300 python3 -u -m pytest tests/test_c3_batch_gpu.py tests/test_match_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest_$tc.log 2>&1
  rc=$?; echo "TC=$tc"; tail -1 $O/pytest_$tc.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest_$tc.log | head -20; exit $rc; }
done
for tc in 256 512 1024; do
  for pass in stats fetch write; do
    case $pass in stats) a="--stats";; fetch) a="--pmc FETCH_SIZE";; write) a="--pmc WRITE_SIZE";; esac
    ORBHIP_MATCH_TC=$tc timeout -s KILL 120 rocprofv3 --kernel-trace $a --output-format csv -d $O/tc${tc}_$pass -o run -- python3 tools/pmc_workload.py c3 > $O/tc${tc}_$pass.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "tc $tc $pass rc=$rc"; tail -5 $O/tc${tc}_$pass.log; exit 1; }
  done
  python3 tools/prof_summary.py traffic "$(ls $O/tc${tc}_fetch/*counter_collection.csv | head -1)" "$(ls $O/tc${tc}_write/*counter_collection.csv | head -1)" $O/traffic_tc$tc.json c3 > /dev/null || exit 1
  python3 - <<PY
import json, csv, glob, collections
t=json.load(open("$O/traffic_tc$tc.json"))["kernels"]
rows=list(csv.DictReader(open(glob.glob("$O/tc${tc}_stats/*kernel_trace.csv")[0])))
agg=collections.defaultdict(list)
for r in rows:
    n=r['Kernel_Name'].split('(')[0].replace('orbhip::','')
    agg[n.split('<')[0]].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
print("TC=$tc", {k: round(sum(v)/len(v),1) for k,v in agg.items() if 'match' in k}, {k: v['hbm_bytes_per_launch'] for k,v in t.items() if 'match' in k or 'octree' in k}, 'octree us', round(sum(agg['k_octree'])/len(agg['k_octree']),1))
PY
done
