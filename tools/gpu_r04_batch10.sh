# Round-4 batch 10: rocprofv3 kernel trace + stats of the headline bench command (two frames in
# flight) and of its single-frame form, and the trace launches' overlap.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04
mkdir -p $O
for fif in 2 1; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_fif$fif -o run -- python3 bench.py --steps 20 --warmup 5 --frames-in-flight $fif --no-cpu-baseline --c5-frames 0 --no-streaming > $O/prof_fif$fif.json 2> $O/prof_fif$fif.err || { tail -20 $O/prof_fif$fif.err; exit 1; }
  skip=0; [ $fif = 2 ] && skip=25  # the single-frame leg (W + K launches) follows the timed steps
  python3 tools/trace_overlap.py $(ls $O/prof_fif$fif/*kernel_trace.csv | head -1) 20 $skip > $O/trace_overlap_fif$fif.json || exit 1
  python3 -c "import json;d=json.load(open('$O/trace_overlap_fif$fif.json'));print($fif, d['duration_ms'], d['gap_to_previous_end_ms'], d['end_to_end_period_ms'])"
done
