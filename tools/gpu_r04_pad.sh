# r04: where the C4 slot-boundary gap sits (an empty kernel at each slot start; the unfused trial)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_pad
mkdir -p $O
ORBHIP_BA_PAD=1 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/pad -o c4 -- python3 tools/time_ba.py 5 > $O/pad.log 2>&1 || { tail $O/pad.log; exit 1; }
ORBHIP_BA_FUSED=0 timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/unf -o c4 -- python3 tools/time_ba.py 5 > $O/unf.log 2>&1 || { tail $O/unf.log; exit 1; }
