# Round-6 shared-grid pass: the frames-in-flight and bench GPU tests, the default bench line, and a
# rocprofv3 kernel trace of the same command (tools/grid_overlap.py: the timed launches side by side).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06
TAG=${TAG:-grid}
mkdir -p $O
timeout -k 10 600 python -u tools/run_gpu_suite.py tests/test_gpu_frames.py tests/test_gpu_bench.py -m gpu -x -v --timeout 300 \
    --timeout-method thread > $O/pytest_gpu_${TAG}.log 2>&1 || { tail -30 $O/pytest_gpu_${TAG}.log; exit 1; }
tail -3 $O/pytest_gpu_${TAG}.log
timeout -k 10 300 python -u bench.py > $O/bench_${TAG}.json 2> $O/bench_${TAG}.err || { tail -20 $O/bench_${TAG}.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_${TAG} -o run -- \
    python3 bench.py --no-cpu-baseline --c5-frames 0 --no-streaming > $O/prof_${TAG}.json 2> $O/prof_${TAG}.err || { tail -20 $O/prof_${TAG}.err; exit 1; }
f=$(find $O/prof_${TAG} -name 'run_kernel_trace.csv' | head -n 1)
python3 tools/grid_overlap.py $f $O/prof_${TAG}.json > $O/grid_overlap_${TAG}.json || exit 1
cat $O/grid_overlap_${TAG}.json
python3 -c "import json;d=json.loads(open('$O/bench_${TAG}.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['single_frame']['value'], d['config']['trace_grid_cus'], d['roofline']['frac'])"
