# A/B of design-experiment libraries on the small-launch shapes (C2: 100K x 8; one 8-GPU rank's C5
# shard: 125K x 16) and C3 as the control: trace time (median of 11) and IR checksum per library.
#   LIBS="tag1 tag2" bash tools/gpu_ab_small.sh      (the product libarx.so runs first)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r04}
mkdir -p gpurun_out/$RD
OUT=gpurun_out/$RD/ab_small_${TAG:-x}.log
for round in 1 2; do
  for shape in "100,100,10 8" "50,50,50 16" "100,100,100 16"; do
    set -- $shape
    RAYS=$1 BOUNCES=$2 timeout -k 10 120 python tools/trace_once.py 12 | sed "s/^/$1x$2 /" | tee -a $OUT || exit 1
    for t in $LIBS; do
      RAYS=$1 BOUNCES=$2 ARX_LIB=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$t.so timeout -k 10 120 python tools/trace_once.py 12 | sed "s/^/$1x$2 /" | tee -a $OUT || exit 1
    done
  done
done
