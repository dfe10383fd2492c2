# Round-4 batch 11: up to three frames in flight -- the frames tests, C2 / C3 bench lines with 2 and
# 3 frames (driver K/W), then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 python -u tools/run_gpu_suite.py tests/test_gpu_frames.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_frames_r04p.log 2>&1 || { tail -40 $O/pytest_frames_r04p.log; exit 1; }
grep -E "passed|failed" $O/pytest_frames_r04p.log | tail -1
for wl in c2 c3; do for f in 2 3; do
  timeout -k 10 300 python3 bench.py --workload $wl --frames-in-flight $f --steps 20 --warmup 5 --no-cpu-baseline --c5-frames 0 --no-streaming > $O/bench_${wl}_fif${f}_r04p.json 2> $O/bench_${wl}_fif${f}_r04p.err || { tail -5 $O/bench_${wl}_fif${f}_r04p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${wl}_fif${f}_r04p.json'));print('$wl', $f, d['value'], d['ms_per_step'], d['single_frame']['value'])"
done; done
TAG=r04p bash tools/gpu_suite_only.sh > /dev/null || { tail -30 $O/pytest_gpu_r04p.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu_r04p.log | tail -1
