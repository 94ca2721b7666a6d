# r06: C4 LBA knobs A/B on one box (k_ba_lin pose work-groups, Schur chunk), then the BA tests
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_ba_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r06_c4ab_tests.log 2>&1
rc=$?; tail -2 gpurun_out/r06_c4ab_tests.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for cfg in "ORBHIP_LIN_PPW=4" "ORBHIP_LIN_PPW=1" "ORBHIP_LIN_PPW=1 ORBHIP_SCHUR_CHUNK=2" "ORBHIP_LIN_PPW=1 ORBHIP_SCHUR_CHUNK=8"; do
  echo "== $cfg: $(env $cfg timeout -k 10 60 python3 tools/time_ba.py 50 2>&1 | grep -v amdgpu.ids | tail -1)"
done
done
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06_c4trace2 -o run -- python3 tools/pmc_workload.py c4lba > gpurun_out/r06_c4trace2.log 2>&1 || { tail -5 gpurun_out/r06_c4trace2.log; exit 1; }
python3 tools/trace_window.py "$(ls gpurun_out/r06_c4trace2/*kernel_trace.csv | head -1)" k_ba_ctl_init 1 2>&1 | head -10
