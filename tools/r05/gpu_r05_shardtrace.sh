# r05: kernel trace of the 8 in-process segment shards of the C5 GBA (the per-rank pieces of the
# modelled 8-rank trial)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r05_shardtrace
mkdir -p $O
timeout -k 10 180 python3 -u tools/time_shard_nd.py 8 > $O/time.log 2>&1 || { tail -5 $O/time.log; exit 1; }
grep -v amdgpu $O/time.log
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o sh -- python3 -u tools/time_shard_nd.py 8 > $O/tr.log 2>&1 || { tail -5 $O/tr.log; exit 1; }
python3 tools/trace_window.py "$(ls $O/tr/*kernel_trace.csv | head -1)" k_ba_sh_init 1 --grid | head -50
