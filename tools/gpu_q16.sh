# Quantized-node (QNode2) trace variants vs the default, plus utilisation counters.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_variants.py 772,900,901,902,903,904,905,906,907,908,772 > gpurun_out/q16_variants.log 2>&1 || { tail -20 gpurun_out/q16_variants.log; exit 1; }
cat gpurun_out/q16_variants.log
UTIL_VARIANT=779 timeout -k 10 120 python -u tools/trace_util.py > gpurun_out/q16_util779.log 2>&1 || { tail -20 gpurun_out/q16_util779.log; exit 1; }
UTIL_VARIANT=909 timeout -k 10 120 python -u tools/trace_util.py > gpurun_out/q16_util909.log 2>&1 || { tail -20 gpurun_out/q16_util909.log; exit 1; }
cat gpurun_out/q16_util779.log gpurun_out/q16_util909.log
