# rocprofv3 kernel trace + stats of the driver's own bench command (K = 20, W = 5) on one MI355X, and
# the trace launches' legs (tools/grid_overlap.py: the timed two-frame launches side by side, the
# kernel-times leg against the line's HIP events).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r06
TAG=${TAG:-drv}
mkdir -p $O
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/prof_${TAG} -o run -- \
    python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_${TAG}.json 2> $O/prof_${TAG}.err || { tail -20 $O/prof_${TAG}.err; exit 1; }
f=$(find $O/prof_${TAG} -name 'run_kernel_trace.csv' | head -n 1)
python3 tools/grid_overlap.py $f $O/prof_${TAG}.json > $O/grid_overlap_${TAG}.json || exit 1
cat $O/grid_overlap_${TAG}.json
