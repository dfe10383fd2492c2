# A/B of convolution design-experiment libraries (build.py --exp TAG -D ARX_CONV_...) on C3.
#   LIBS="tag1 tag2" bash tools/gpu_conv_ab.sh      (the product libarx.so runs first and last)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
OUT=gpurun_out/conv_ab_${TAG:-x}.log
timeout -k 10 120 python tools/conv_once.py 21 | tee -a $OUT || exit 1
for t in $LIBS; do
  ARX_LIB=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$t.so timeout -k 10 120 python tools/conv_once.py 21 | tee -a $OUT || exit 1
done
timeout -k 10 120 python tools/conv_once.py 21 | tee -a $OUT || exit 1
