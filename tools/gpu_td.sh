set -o pipefail
cd "$GRAFT_REPO_ROOT" && mkdir -p gpurun_out
timeout -k 10 120 ./tools/experiments/td_microbench > gpurun_out/td_microbench.log 2>&1 && cat gpurun_out/td_microbench.log &&
ARX_LIB=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_count.so timeout -k 10 120 python tools/trace_counts.py > gpurun_out/trace_counts.json && cat gpurun_out/trace_counts.json
