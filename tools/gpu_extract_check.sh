set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_extract_gpu.py tests/test_golden.py tests/test_match_gpu.py -x -q -m gpu > gpurun_out/ext_tests.log 2>&1; rc=$?; tail -4 gpurun_out/ext_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 300 > gpurun_out/bench_cone.log 2>&1 && tail -1 gpurun_out/bench_cone.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cone', d['value'], d['roofline']['stage_avg_ms_calibration'])"
ORBHIP_NO_CONE=1 timeout -k 10 300 python bench.py --no-cpu --no-extra --steps 300 > gpurun_out/bench_nocone.log 2>&1 && tail -1 gpurun_out/bench_nocone.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cascade', d['value'], d['roofline']['stage_avg_ms_calibration'])"
