# Quick A/B of experiment libraries against the product (C3 and C2 trace, tools/gpu_ab_libs.sh);
# LIBS / SHAPES / OUT from the environment.  Output under gpurun_out/r03/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
OUT=${OUT:-ab_quick}
LIBS="$LIBS" SHAPES="${SHAPES:-c3 c2}" bash tools/gpu_ab_libs.sh > gpurun_out/r03/$OUT.txt 2>&1 || { tail -n 20 gpurun_out/r03/$OUT.txt; exit 1; }
cat gpurun_out/r03/$OUT.txt
