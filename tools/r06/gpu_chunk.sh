# r06: C4 LBA against the lone problem's Schur chunk (pairs per work item), alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
for rep in 1 2 3; do
  for c in 1 2 3 4; do
    echo -n "chunk=$c  "; ORBHIP_SCHUR_CHUNK=$c timeout -k 10 60 python3 tools/time_ba.py 50 2>&1 | grep LBA || exit 1
  done
done
for c in 2 4; do echo -n "GBA chunk=$c  "; ORBHIP_SCHUR_CHUNK=$c timeout -k 10 120 python3 tools/time_gba.py 2>&1 | grep GBA || exit 1; done
