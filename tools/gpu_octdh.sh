# k_octree device trace (C2 level 0 phases) per division engine / pyramid depth cap, then the
# C2 stage averages of the bench (k_octree over 300 frames).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mode in auto sweep dh6; do
  case $mode in sweep) ev="ORBHIP_OCTREE_SWEEP=1";; dh6) ev="ORBHIP_OCTREE_DH=6";; auto) ev="X=1";; esac
  env $ev ORBHIP_TRACE_BLOCK=0 timeout -k 10 120 python3 -u tools/trace_c2.py > gpurun_out/trace_$mode.log 2>&1 || exit 1
  echo "$mode"; grep -A1 k_octree gpurun_out/trace_$mode.log
  env $ev timeout -k 10 120 python3 bench.py --no-cpu --no-extra --steps 100 > gpurun_out/bench_$mode.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/bench_$mode.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$mode', d['value'], d['batch1_frames_per_s'], d['roofline']['kernel'], d['roofline']['stage_avg_ms_calibration'])"
done
