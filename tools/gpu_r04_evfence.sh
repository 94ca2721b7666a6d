# r04: BA slot pacing (events without the system fence, then progress words): BA tests, LBA/GBA timing, C4 trace gaps
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=${O:-gpurun_out/r04_evf}
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_concurrent_gpu.py tests/test_nd_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_sharded_nd_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
timeout -k 10 120 python3 tools/time_ba.py 20 > $O/lba.log 2>&1 || exit 1
grep LBA $O/lba.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o c4 -- python3 tools/time_ba.py 5 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
python3 tools/ba_trace_summary.py "$(ls $O/prof/*kernel_trace.csv | head -1)" | head -12
timeout -k 10 120 python3 -u tools/time_gba.py > $O/gba.log 2>&1 && grep GBA $O/gba.log
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 -u tools/time_gba.py > $O/gba_timing.log 2>&1 && grep "timing B=1" $O/gba_timing.log | tail -2
ORBHIP_BA_TIMING=1 timeout -k 10 120 python3 tools/time_ba.py 3 > $O/lba_timing.log 2>&1 && grep "timing B=1" $O/lba_timing.log | tail -2
