# r03 work loop: selected GPU tests, then timing tools (each step bounded, stops at the first failure)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_work.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_work.log; [ $rc -eq 0 ] || exit $rc
for t in $TOOLS; do
  echo "== $t"
  timeout -k 10 150 python3 $t > gpurun_out/tool.log 2>&1 || { tail -20 gpurun_out/tool.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/tool.log | tail -${TAILN:-12}
done
