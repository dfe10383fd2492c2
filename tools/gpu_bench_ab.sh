# A/B of design-experiment libraries in the bench's own context (tools/bench_lib.py):
#   LIBS="tag1 tag2" bash tools/gpu_bench_ab.sh   (the product libarx.so runs first and last)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
O=gpurun_out/bench_ab_${TAG:-x}.log
P=$GRAFT_REPO_ROOT/audiorenderingv2_amd/libarx.so
for lib in $P $(for t in $LIBS; do echo $GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$t.so; done) $P; do
  timeout -k 10 200 python tools/bench_lib.py $lib --no-cpu-baseline --c5-frames 0 --steps 20 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib)', 'conv_us', round(d['phases_ms_rank0']['ir_spectra_and_convolution']*1e3,1), 'trace_ms', round(d['phases_ms_rank0']['trace_kernel'],4), 'step_ms', round(d['ms_per_step'],4))" | tee -a $O || exit 1
done
