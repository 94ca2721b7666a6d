# r05: kernel traces of the C5 GBA and the C4 LBA (per-kernel time per LM trial)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_trace}
mkdir -p $O
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/gba -o gba -- python3 -u tools/time_gba.py > $O/gba.log 2>&1 || { tail -5 $O/gba.log; exit 1; }
grep GBA $O/gba.log
python3 tools/trace_window.py "$(ls $O/gba/*kernel_trace.csv | head -1)" k_ba_ctl_init 1 | head -40
timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/lba -o lba -- python3 -u tools/pmc_workload.py c4lba > $O/lba.log 2>&1 || { tail -5 $O/lba.log; exit 1; }
python3 tools/trace_window.py "$(ls $O/lba/*kernel_trace.csv | head -1)" k_ba_ctl_init 1 | head -40
