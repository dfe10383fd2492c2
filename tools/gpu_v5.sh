# v5 (branch-minimal steps) and quantized variants on the SBVH default, then the parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_variants.py 863,772,900,920,921,922,923,924,925,926,927,928,929 > gpurun_out/v5_variants.log 2>&1 || { tail -20 gpurun_out/v5_variants.log; exit 1; }
cat gpurun_out/v5_variants.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/v5_parity.log 2>&1 || { tail -30 gpurun_out/v5_parity.log; exit 1; }
tail -3 gpurun_out/v5_parity.log
