# r04: C4 slot-boundary gap against the number of slots in flight (ORBHIP_BA_DEPTH)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_depth
mkdir -p $O
for D in 2 3 4; do
  ORBHIP_BA_DEPTH=$D timeout -k 10 120 python3 tools/time_ba.py 20 > $O/lba_$D.log 2>&1 || exit 1
  echo "depth $D: $(grep LBA $O/lba_$D.log)"
done
for D in 2 4; do
  ORBHIP_BA_DEPTH=$D timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $O/prof$D -o c4 -- python3 tools/time_ba.py 5 > $O/prof$D.log 2>&1 || { tail $O/prof$D.log; exit 1; }
done
