# C2 headline (16 cameras) and batch-1 figure, repeated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 100 python3 bench.py --no-cpu --no-extra --steps 200 "$@" > gpurun_out/shape_$name.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/shape_$name.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$name', d['value'], d['batch1_frames_per_s'], c['one_camera_8_in_flight_frames_per_s'], d['roofline']['stage_avg_ms_calibration'])"
}
run a
run b
run c
