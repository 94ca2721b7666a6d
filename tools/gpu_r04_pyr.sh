# r04: batch pyramid engines at C3 after the readfirstlane fix: the k_resize cascade (default),
# k_resize_bands (ORBHIP_RZ_BANDS=n) and k_pyr_flow (ORBHIP_RZ_FLOW=1), kernel traces of the C3
# batch workload; parity of the bands / flow engines first
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_pyr
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_extract_gpu.py tests/test_c3_batch_gpu.py -k "cascade or flow or c3_batch_vs" -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for cfg in "X=0" "ORBHIP_RZ_FLOW=1" "ORBHIP_RZ_BANDS=16" "ORBHIP_RZ_BANDS=64"; do
  tag=$(echo $cfg | tr '=' '_')
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$tag -o c3 -- python3 tools/pmc_workload.py c3 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  python3 - <<PY
import csv, glob, collections
rows=list(csv.DictReader(open(glob.glob("$O/$tag/*kernel_trace.csv")[0])))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
agg=collections.defaultdict(list)
for r in rows:
    n=r['Kernel_Name'].split('(')[0].replace('orbhip::','')
    agg[n].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
# pyramid per batch: sum of pyramid kernels / 4 batches
pyr=sum(sum(v) for k,v in agg.items() if k in ('k_resize','k_resize_bands','k_pyr_flow'))/4
print("$cfg", 'pyramid kernels per batch us', round(pyr,1), {k:(len(v), round(sum(v)/len(v),1)) for k,v in agg.items() if k.startswith('k_')})
PY
done
