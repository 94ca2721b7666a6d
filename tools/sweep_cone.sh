cd "${GRAFT_REPO_ROOT:-/root/repo}"
for ts in 16 12 10 8; do
  echo "tile $ts"; ORBHIP_CONE_TILE=$ts timeout -k 10 100 python tools/trace_c2.py 2>&1 | grep -v amdgpu.ids | head -1
  ORBHIP_CONE_TILE=$ts timeout -k 10 100 python bench.py --no-cpu --no-extra --steps 300 | cut -c 90-130
done
