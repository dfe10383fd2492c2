set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
TAG=r03k
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r03/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/r03/pytest_gpu_$TAG.log; exit 1; }
tail -3 gpurun_out/r03/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/r03/smoke_$TAG.log; exit 1; }
timeout -k 10 400 python3 bench.py > gpurun_out/r03/bench_$TAG.json 2> gpurun_out/r03/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/r03/bench_$TAG.err; exit 1; }
cat gpurun_out/r03/bench_$TAG.json
