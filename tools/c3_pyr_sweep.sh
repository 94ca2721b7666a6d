# C3 pyramid stage: the batch cone at several tile edges and the k_resize-only cascade
# (rocprofv3 kernel trace of 4 C3 batches each; per-kernel durations of the last batch)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/c3sweep
for cfg in ${CFGS:-b8 b16 b32 b64 resize}; do
  case $cfg in
    resize) envs="ORBHIP_RZ_BANDS=0";;
    b*) envs="ORBHIP_RZ_BANDS=${cfg#b}";;
    w*) t=${cfg#w}; envs="ORBHIP_CONE_HI=1 ORBHIP_CONE_HI_TILE=${t%_*} ORBHIP_CONE_HI_THREADS=${t#*_}";;
    t*) envs="ORBHIP_CONE_HI=1 ORBHIP_CONE_HI_TILE=${cfg#t}";;
  esac
  env $envs timeout -k 10 100 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/c3sweep/$cfg -o c3 \
      -- python3 tools/pmc_workload.py c3 > gpurun_out/c3sweep/$cfg.log 2>&1 || { tail -5 gpurun_out/c3sweep/$cfg.log; exit 1; }
  python3 - "$cfg" <<'PY'
import csv, sys, glob
f = glob.glob(f"gpurun_out/c3sweep/{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
last = [r for r in rows if "k_resize" in r["Kernel_Name"] or "k_pyr_cone" in r["Kernel_Name"]]
k = last[-(7 if sys.argv[1] == "resize" else 3):]   # the last batch's pyramid launches
span = (int(k[-1]["End_Timestamp"]) - int(k[0]["Start_Timestamp"])) / 1e3
print(sys.argv[1], f"stage {span:.1f} us:", " ".join(f"{r['Kernel_Name'].split('(')[0].split('::')[-1]}:{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3:.1f}" for r in k))
PY
done
