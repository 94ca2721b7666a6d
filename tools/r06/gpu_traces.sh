# r06: BA kernel traces per LM trial (profiles/r06_ba_traces.md): C5 GBA one GPU, C4 LBA, and the
# 8 in-process shards of both sharded forms (segments; landmark shards with the summed S dissected)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
tw() { python3 tools/trace_window.py "$(ls gpurun_out/$1/*kernel_trace.csv | head -1)" "${@:2}"; }
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_tr_gba -o run -- python3 tools/time_gba.py > gpurun_out/r06_tr_gba.log 2>&1 || exit 1
echo "## C5 GBA"; grep GBA gpurun_out/r06_tr_gba.log; tw r06_tr_gba k_ba_ctl_init 1
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_tr_lba -o run -- python3 tools/pmc_workload.py c4lba > gpurun_out/r06_tr_lba.log 2>&1 || exit 1
echo "## C4 LBA"; tw r06_tr_lba k_ba_ctl_init 1
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r06_tr_shard -o run -- python3 tools/time_shard_nd.py 8 > gpurun_out/r06_tr_shard.log 2>&1 || exit 1
echo "## shards"; grep -v amdgpu gpurun_out/r06_tr_shard.log | grep ms
echo "### 8 segment shards"; tw r06_tr_shard k_ba_sh_init 5 --grid
echo "### 8 landmark shards, summed S dissected"; tw r06_tr_shard k_ba_sh_init 3 --grid
