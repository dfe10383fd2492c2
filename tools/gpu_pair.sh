# Pair-cooperative fetch (940-945) vs the default (921), then the parity tests.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/trace_variants.py 921,940,941,942,943,944,945,932,921 > gpurun_out/pair_variants.log 2>&1 || { tail -20 gpurun_out/pair_variants.log; exit 1; }
cat gpurun_out/pair_variants.log
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/pair_parity.log 2>&1 || { tail -30 gpurun_out/pair_parity.log; exit 1; }
tail -3 gpurun_out/pair_parity.log
