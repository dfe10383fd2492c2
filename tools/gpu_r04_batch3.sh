# Round-4 batch 3: the pass-C occupancy fix -- convolution A/B against the previous product
# (libarx_base) and 8-column pass C (tcc8), phases of the fixed build; the C2 latency floor; then the
# GPU suite with the native crash tracer.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS="base tcc8" TAG=r04h bash tools/gpu_conv_ab.sh > /dev/null || exit 1
cat gpurun_out/r04/conv_ab_r04h.log
TAG=r04h bash tools/gpu_conv_phases.sh || exit 1
timeout -k 10 300 python3 tools/c2_floor.py gpurun_out/r04/c2_floor.json > gpurun_out/r04/c2_floor.log 2>&1 || { tail -20 gpurun_out/r04/c2_floor.log; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r04/c2_floor.json'));print({k:v for k,v in d.items() if k!='slowest_waves_remeasured_ms'})"
TAG=r04h bash tools/gpu_suite_only.sh
