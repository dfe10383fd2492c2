# Full GPU round: tests, bench, rocprof kernel stats, PMC traffic of the bench's trace kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r01d}
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -3 gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run -- python3 bench.py --no-cpu-baseline --c5-frames 0 > gpurun_out/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
tail -2 gpurun_out/prof_$TAG.log
mkdir -p gpurun_out/pmc_traffic_$TAG
for grp in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_traffic_$TAG/$grp" -o p -- python3 tools/trace_once.py 2 > gpurun_out/pmc_traffic_$TAG/$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/pmc_traffic_$TAG/$grp.log; exit 1; }
done
python tools/make_traffic.py gpurun_out/pmc_traffic_$TAG c3 gpurun_out/trace_traffic_$TAG.json
# pipeline / memory counters of the product trace kernel
rm -rf gpurun_out/pmcs && CONFIGS=prod bash tools/gpu_pmc_state.sh > gpurun_out/pmc_state_$TAG.txt 2>&1 || { echo "pmc state failed"; tail -20 gpurun_out/pmc_state_$TAG.txt; exit 1; }
tail -40 gpurun_out/pmc_state_$TAG.txt
