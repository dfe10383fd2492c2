# Round-4 measurement batch: convolution phases (product and 2-pair pass B), convolution A/B, the
# small-launch fused-step A/B, then the regular round (smoke, bench, GPU suite with the crash tracer).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r04f bash tools/gpu_conv_phases.sh || exit 1
ARX_LIB=tools/experiments/lib/libarx_cprofbm2.so TAG=r04f_bm2 bash tools/gpu_conv_phases.sh || exit 1
LIBS="bm2 bm4" TAG=r04f bash tools/gpu_conv_ab.sh > /dev/null || exit 1
tail -n 9 gpurun_out/r04/conv_ab_r04f.log
LIBS="fuse" TAG=r04f bash tools/gpu_ab_small.sh > /dev/null || exit 1
cut -c1-120 gpurun_out/r04/ab_small_r04f.log
TAG=r04f bash tools/gpu_round.sh
