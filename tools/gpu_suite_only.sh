# The GPU test suite alone, in one process, with the native crash tracer (tools/run_gpu_suite.py);
# log under gpurun_out/$RD/pytest_gpu_$TAG.log.  K= restricts pytest (-k expression).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r04}
O=gpurun_out/$RD
TAG=${TAG:-x}
mkdir -p $O
timeout -k 10 900 python -u tools/run_gpu_suite.py tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -n 45 $O/pytest_gpu_$TAG.log
exit $rc
