# r04: BA after the once-per-slot stop relay: BA tests, single and batched C4, GBA
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_batch
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py tests/test_ba_concurrent_gpu.py tests/test_nd_gpu.py tests/test_ba_sharded_gpu.py tests/test_ba_sharded_nd_gpu.py -m gpu -q -x --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -1 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/pytest.log | head -20; exit $rc; }
for i in 1 2; do timeout -k 10 180 python3 tools/time_ba.py 20 256 > $O/lba_$i.log 2>&1 || exit 1; grep LBA $O/lba_$i.log; done
timeout -k 10 120 python3 -u tools/time_gba.py > $O/gba.log 2>&1 && grep GBA $O/gba.log
