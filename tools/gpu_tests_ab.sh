# GPU test suite (one process) then an A/B of experiment libraries against the product;
# TAG names the test log, LIBS / OUT the A/B (tools/gpu_ab_quick.sh).  Output under gpurun_out/r03/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
TAG=${TAG:-x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -n 30 gpurun_out/r03/pytest_gpu_$TAG.log; exit 1; }
tail -n 2 gpurun_out/r03/pytest_gpu_$TAG.log
[ -z "$LIBS" ] || LIBS="$LIBS" OUT="$OUT" bash tools/gpu_ab_quick.sh
