# r04: ND back-substitution change: ND / sharded-ND / BA parity tests, probe timings, C5 GBA time,
# and a kernel trace of the one-GPU C5 GBA
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04_nd2}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_nd_gpu.py tests/test_ba_sharded_nd_gpu.py tests/test_ba_gpu.py tests/test_ba_concurrent_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 -u tools/probe_nd.py > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
cat $O/probe.log
timeout -k 10 120 python3 -u tools/time_gba.py > $O/gba.log 2>&1 || exit 1
grep GBA $O/gba.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o gba -- python3 -u tools/time_gba.py > $O/prof.log 2>&1 || { tail -5 $O/prof.log; exit 1; }
python3 tools/ba_trace_summary.py "$(ls $O/prof/*kernel_trace.csv | head -1)" | head -16
