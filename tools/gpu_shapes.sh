# C2 16-camera headline under launch knobs (kernels / packets per frame vs throughput).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {
  name=$1; shift
  env "$@" timeout -k 10 100 python3 bench.py --no-cpu --no-extra --steps 200 ${BENCH_ARGS:-} > gpurun_out/shape_$name.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/shape_$name.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config']; print('$name', d['value'], d['batch1_frames_per_s'], c['one_camera_8_in_flight_frames_per_s'])"
}
run default X=1
run noev ORBHIP_FE_NOEV=1
run default2 X=1
run noev2 ORBHIP_FE_NOEV=1
