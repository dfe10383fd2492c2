# A/B of design-experiment libraries on the C3 (and C2-shaped) trace: each lib rendered in turn,
# twice, median trace ms of 6 renders (tools/trace_once.py).  LIBS="prod dyn32 ..." (prod = the
# product library), SHAPES="c3 c2".
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for round in 1 2; do
  for shape in ${SHAPES:-c3}; do
    if [ "$shape" = c2 ]; then export RAYS=100,100,10 BOUNCES=8; else export RAYS=100,100,100 BOUNCES=16; fi
    for lib in ${LIBS:-prod}; do
      if [ "$lib" = prod ]; then L=""; else L=tools/experiments/lib/libarx_$lib.so; fi
      printf "%s %s " "$shape" "$lib"
      ARX_LIB=$L timeout -k 10 120 python tools/trace_once.py ${N:-6} || exit 1
    done
  done
done
