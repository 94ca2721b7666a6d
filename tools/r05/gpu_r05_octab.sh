# r05: octree A/B on the C2 section, alternating runs: main (wave-0 MAIN + register FINAL, 512 threads),
# nofinal (wave-0 MAIN only), octbase (r04's block loop at 1024 threads)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_octab
mkdir -p $O
for i in 1 2 3; do
  for v in main nofinal octbase; do
    unset ORBHIP_LIB ORBHIP_OCT_NT
    [ $v = main ] || export ORBHIP_LIB=tools/ubench/ab/liborbhip_$v.so
    [ $v = octbase ] && export ORBHIP_OCT_NT=1024
    timeout -k 10 300 python3 -u bench.py --no-extra --no-cpu > $O/bench_${v}_$i.json 2> $O/bench_${v}_$i.err || { tail -5 $O/bench_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/bench_${v}_$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['batch1_latency_ms'], d['roofline']['stage_avg_ms']['k_octree'])"
  done
done
