# A/B of design-experiment libraries (build.py --exp TAG -D...) on the C3 trace workload.
#   LIBS="tag1 tag2" bash tools/gpu_ab.sh      (the product libarx.so always runs first)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/ab_${TAG:-x}.log
timeout -k 10 120 python tools/trace_once.py 12 | tee -a $OUT || exit 1
if [ -d tools/experiments/old ]; then  # an older tree's package + library (A/B baseline)
  ARX_PKG_ROOT=$GRAFT_REPO_ROOT/tools/experiments/old timeout -k 10 120 python tools/trace_once.py 12 | tee -a $OUT || exit 1
fi
for t in $LIBS; do
  ARX_LIB=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$t.so timeout -k 10 120 python tools/trace_once.py 12 | tee -a $OUT || exit 1
done
