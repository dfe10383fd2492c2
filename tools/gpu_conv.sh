# Convolution timing on the bench workload, then the convolution / live / export parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --no-cpu-baseline --c5-frames 0 --steps 10 > gpurun_out/conv_bench.json 2> gpurun_out/conv_bench.err || { tail -20 gpurun_out/conv_bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/conv_bench.json')); print(d['phases_ms_rank0'], d['value'], d['convolved_frames_per_s'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_conv" -o run -- python3 bench.py --no-cpu-baseline --c5-frames 0 --steps 5 > gpurun_out/prof_conv.log 2>&1 || { tail -20 gpurun_out/prof_conv.log; exit 1; }
head -8 gpurun_out/prof_conv/run_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_live.py tests/test_gpu_app.py -x -q -k "conv or live or export or app" --timeout 300 --timeout-method thread > gpurun_out/conv_parity.log 2>&1 || { tail -30 gpurun_out/conv_parity.log; exit 1; }
tail -3 gpurun_out/conv_parity.log
