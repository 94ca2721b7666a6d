# r05: cone threads per tile A/B (ORBHIP_CONE_NT 1024 / 512 / 256) on the C2 section, alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_conent
mkdir -p $O
ORBHIP_CONE_NT=256 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_extract_gpu.py tests/test_frontend.py > $O/pytest.log 2>&1 || { tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
  for nt in 1024 512 256; do
    ORBHIP_CONE_NT=$nt timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${nt}_$i.json 2> $O/bench_${nt}_$i.err || { tail -5 $O/bench_${nt}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${nt}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('nt=$nt', d['value'], d['batch1_latency_ms'], r['avg_launch_ms'], r['stage_avg_ms_one_frame_stream']['pyramid (k_pyr_cone | 7x k_resize)'])"
  done
done
