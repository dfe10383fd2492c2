# Octant copies of the quantized nodes (932-937) vs the default (921), SBVH parameter sweep, parity.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_variants.py 921,932,933,934,935,936,937,921 > gpurun_out/oct_variants.log 2>&1 || { tail -20 gpurun_out/oct_variants.log; exit 1; }
cat gpurun_out/oct_variants.log
: > gpurun_out/sbvh_sweep.log
for cfg in 0 1e-3,3,32,4,1,1 1e-3,3,32,4,1,2 1e-3,3,32,4,1,3 1e-3,3,32,2,1,1 1e-3,3,32,3,1,1 1e-3,3,32,6,1,1 1e-4,3,32,4,1,1 1e-2,3,32,4,1,1 1e-3,3,16,4,1,1 1e-3,3,64,4,1,1; do
  echo "ARX_SBVH=$cfg" >> gpurun_out/sbvh_sweep.log
  ARX_SBVH=$cfg timeout -k 10 120 python -u tools/trace_variants.py 921,932 >> gpurun_out/sbvh_sweep.log 2>&1 || { tail -20 gpurun_out/sbvh_sweep.log; exit 1; }
done
cat gpurun_out/sbvh_sweep.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/oct_parity.log 2>&1 || { tail -30 gpurun_out/oct_parity.log; exit 1; }
tail -3 gpurun_out/oct_parity.log
