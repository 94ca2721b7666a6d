# r04: where the persistent Cholesky's chain spends an interval (raw per-interval cycles saved),
# the C4 / C5 solve times, and a kernel trace of the single C4 LBA.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_chain
export ORBHIP_PROBE_SAVE=gpurun_out/r04_chain
timeout -k 10 120 python3 -u tools/probe_cholesky_dag.py 294:dense 2394:loop 2394:dense 912:loop > gpurun_out/r04_chain/probe.log 2>&1 || { tail -20 gpurun_out/r04_chain/probe.log; exit 1; }
cat gpurun_out/r04_chain/probe.log
timeout -k 10 120 python3 -u tools/time_ba.py 20 > gpurun_out/r04_chain/time_ba.log 2>&1 || exit 1
cat gpurun_out/r04_chain/time_ba.log
timeout -k 10 180 python3 -u tools/time_gba.py > gpurun_out/r04_chain/time_gba.log 2>&1 || exit 1
cat gpurun_out/r04_chain/time_gba.log
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r04_chain/prof -o c4 -- python3 tools/time_ba.py 5 > gpurun_out/r04_chain/prof.log 2>&1 || { tail gpurun_out/r04_chain/prof.log; exit 1; }
python3 tools/ba_trace_summary.py "$(ls gpurun_out/r04_chain/prof/*kernel_trace.csv | head -1)" | head -30
