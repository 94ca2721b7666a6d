# r04: k_fast_cells threads per cell on the C2 16-camera stream (ORBHIP_FAST_NT pins it; default:
# the front-end's hint, 256 at 8+ cameras), alternating runs
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_fastnt
mkdir -p $O
for nt in 0 128 512 0 128 512; do
  if [ $nt = 0 ]; then E=""; else E="ORBHIP_FAST_NT=$nt"; fi
  env $E timeout -k 10 300 python3 -u bench.py --no-cpu --no-extra > $O/b_$nt.log 2> $O/b_$nt.err || { tail -5 $O/b_$nt.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/b_$nt.log') if l.startswith('{')][-1]); r=d['roofline']
print('fast_nt $nt value', d['value'], 'batch1', d['batch1_latency_ms'], 'fast stage', r['stage_avg_ms']['k_fast_cells'])"
done
