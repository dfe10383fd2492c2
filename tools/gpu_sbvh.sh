# SBVH (spatial splits) vs object-split SAH on the C3 workload, f32 and quantized nodes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_variants.py 772,863,900,901,910,911,912 > gpurun_out/sbvh_off.log 2>&1 || { tail -20 gpurun_out/sbvh_off.log; exit 1; }
cat gpurun_out/sbvh_off.log
ARX_SBVH=1e-3,3 timeout -k 10 300 python -u tools/trace_variants.py 863,901,910,911,912 > gpurun_out/sbvh_on.log 2>&1 || { tail -20 gpurun_out/sbvh_on.log; exit 1; }
cat gpurun_out/sbvh_on.log
ARX_SBVH=1e-3,3 UTIL_VARIANT=909 timeout -k 10 120 python -u tools/trace_util.py > gpurun_out/sbvh_util909.log 2>&1 || { tail -20 gpurun_out/sbvh_util909.log; exit 1; }
cat gpurun_out/sbvh_util909.log
