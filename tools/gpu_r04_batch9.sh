# Round-4 batch 9: the frames-in-flight tests (all trace paths), then smoke, the default bench line,
# the driver's K/W line and the whole GPU suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04
mkdir -p $O
timeout -k 10 300 python -u tools/run_gpu_suite.py tests/test_gpu_frames.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest_frames_r04n.log 2>&1 || { tail -40 $O/pytest_frames_r04n.log; exit 1; }
grep -E "passed|failed" $O/pytest_frames_r04n.log | tail -1
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_r04n_driverkw.json 2> $O/bench_r04n_driverkw.err || { tail -5 $O/bench_r04n_driverkw.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_r04n_driverkw.json'));print(d['value'], d['ms_per_step'], d['single_frame']['value'], d['phases_ms_rank0'], d['roofline']['frac'])"
TAG=r04n bash tools/gpu_round.sh
