set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python tools/trace_phases.py 1:0,2:32,3:32,4:32,6:32,4:16,4:24,4:40,4:48,6:40,8:40,6:48,8:48 > gpurun_out/phases.log 2>&1 || { echo "phases failed"; tail -20 gpurun_out/phases.log; exit 1; }
cat gpurun_out/phases.log
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q > gpurun_out/pytest_parity.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_parity.log; exit 1; }
tail -2 gpurun_out/pytest_parity.log
