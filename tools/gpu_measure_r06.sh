# Round-6 measurement pass: the guarded trace profiles (tools/gpu_profile.sh: bench line, rocprofv3
# kernel stats, PMC traffic, pipeline state, lane counts, vector-memory ceiling) into gpurun_out/r06/,
# then the C3 convolution's PMC traffic (tools/gpu_conv_pmc.sh, guarded by arx_conv_kernel_id) and its
# per-workgroup phases (measurement build libarx_cprof.so, tools/conv_phases.py).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/r06
RD=r06 TAG=${TAG:-r06} bash tools/gpu_profile.sh > gpurun_out/r06/profile_${TAG:-r06}.txt 2>&1 || { tail -20 gpurun_out/r06/profile_${TAG:-r06}.txt; exit 1; }
tail -5 gpurun_out/r06/profile_${TAG:-r06}.txt
bash tools/gpu_conv_pmc.sh > gpurun_out/r06/conv_traffic.json 2> gpurun_out/r06/conv_pmc.err || { tail -20 gpurun_out/r06/conv_traffic.json gpurun_out/r06/conv_pmc.err; exit 1; }
cp -r gpurun_out/conv_pmc/stats gpurun_out/r06/conv_kernel_stats 2>/dev/null
RD=r06 TAG=r06 bash tools/gpu_conv_phases.sh || exit 1
cat gpurun_out/r06/conv_traffic.json
