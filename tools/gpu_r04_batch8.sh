# Round-4 batch 8: frames in flight -- their parity tests first, then the default bench line
# (driver K/W), C2 and C4 lines, then the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 python -u tools/run_gpu_suite.py tests/test_gpu_frames.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_frames_r04m.log 2>&1 || { tail -40 $O/pytest_frames_r04m.log; exit 1; }
tail -n 3 $O/pytest_frames_r04m.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_r04m.json 2> $O/bench_r04m.err || { tail -5 $O/bench_r04m.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_r04m.json 2> $O/bench_c2_r04m.err || { tail -5 $O/bench_c2_r04m.err; exit 1; }
timeout -k 10 400 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --c5-frames 0 > $O/bench_c4_r04m.json 2> $O/bench_c4_r04m.err || { tail -5 $O/bench_c4_r04m.err; exit 1; }
for f in bench_r04m bench_c2_r04m bench_c4_r04m; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['ms_per_step'], d['single_frame'], d['phases_ms_rank0'], d['roofline']['frac'])"; done
TAG=r04m bash tools/gpu_suite_only.sh > /dev/null || { tail -30 $O/pytest_gpu_r04m.log; exit 1; }
grep -E "passed|failed" $O/pytest_gpu_r04m.log | tail -1
