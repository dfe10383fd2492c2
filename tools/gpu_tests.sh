# GPU test suite only (one process), log under gpurun_out/; optional K= pytest -k expression.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-x}
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_gpu_$TAG.log
exit $rc
