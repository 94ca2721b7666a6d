# r04: C3 batches in flight (bench --c3-inflight 4 / 6 / 8, alternating) after the FAST rework
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04_c3inflight
mkdir -p $O
for n in 4 6 8 4 6 8; do
  timeout -k 10 300 python3 -u bench.py --no-cpu --c3-inflight $n --lba-steps 2 --gba-iters 1 > $O/b_$n.log 2> $O/b_$n.err || { tail -5 $O/b_$n.err; exit 1; }
  python3 -c "
import json; d=json.loads([l for l in open('$O/b_$n.log') if l.startswith('{')][-1]); e=d['extra']
print('inflight $n', e['c3_1280x720_b64_extract_match_frames_per_s'], e['c3_one_batch_at_a_time_frames_per_s'])"
done
