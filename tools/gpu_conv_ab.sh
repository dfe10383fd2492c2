# A/B of convolution design-experiment libraries on the C3 convolution (tools/conv_once.py: median of
# 11 runs, IR re-set before each, so the IR spectra are included; checksum of the outputs).
#   LIBS="tag1 tag2" bash tools/gpu_conv_ab.sh      (the product libarx.so runs first)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r04}
mkdir -p gpurun_out/$RD
OUT=gpurun_out/$RD/conv_ab_${TAG:-x}.log
for round in 1 2 3; do
  timeout -k 10 120 python tools/conv_once.py 12 | tee -a $OUT || exit 1
  for t in $LIBS; do
    ARX_LIB=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$t.so timeout -k 10 120 python tools/conv_once.py 12 | tee -a $OUT || exit 1
  done
done
