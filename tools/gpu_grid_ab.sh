# Persistent-grid share x frames in flight, in the bench's own context (design experiment, round 6):
#   RUNS="lib:fif lib:fif ..." (lib = product | an experiment tag) bash tools/gpu_grid_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06
O=gpurun_out/r06/grid_ab_${TAG:-x}.txt
for run in $RUNS; do
  t=${run%%:*}; f=${run##*:}
  if [ "$t" = product ]; then lib=$GRAFT_REPO_ROOT/audiorenderingv2_amd/libarx.so; else lib=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$t.so; fi
  timeout -k 10 200 python tools/bench_lib.py $lib --no-cpu-baseline --c5-frames 0 --no-streaming --steps 30 --frames-in-flight $f ${EXTRA:-} 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t fif $f', 'value %.3e' % d['value'], 'step_ms', round(d['ms_per_step'],4), 'trace_ms', round(d['phases_ms_rank0']['trace_kernel'],4), 'single_frame %.3e' % (d.get('single_frame') or {}).get('value', 0))" | tee -a $O || exit 1
done
