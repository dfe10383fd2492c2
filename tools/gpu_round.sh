set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_c.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_c.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_c.log
timeout -k 10 400 python bench.py > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || { echo "bench failed"; tail -20 gpurun_out/bench_c.err; exit 1; }
cat gpurun_out/bench_c.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_r01c" -o run -- python3 bench.py --no-cpu-baseline --c5-frames 0 > gpurun_out/prof_r01c.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_r01c.log; exit 1; }
tail -2 gpurun_out/prof_r01c.log
