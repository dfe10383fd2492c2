set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -k "wide or variants" > gpurun_out/pytest_wide.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_wide.log; exit 1; }
tail -3 gpurun_out/pytest_wide.log
timeout -k 10 600 python tools/trace_variants.py 0,300,320,321,322,323,324,325,326,327,328,329 > gpurun_out/variants_wide.log 2>&1 || { echo "variants failed"; tail -20 gpurun_out/variants_wide.log; exit 1; }
cat gpurun_out/variants_wide.log
