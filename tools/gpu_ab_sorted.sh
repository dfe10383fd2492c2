set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
LIBS="prod sort6 sort8 sort8s192" SHAPES="c3 c2" bash tools/gpu_ab_libs.sh > gpurun_out/r03/ab_sorted_dirs.txt 2>&1 || { tail -n 20 gpurun_out/r03/ab_sorted_dirs.txt; exit 1; }
cat gpurun_out/r03/ab_sorted_dirs.txt
bash tools/gpu_validate.sh
