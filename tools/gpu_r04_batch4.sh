# Round-4 batch 4: small-launch rays-per-wave A/B (C2, one 8-GPU rank's C5 shard, C3 control), then
# the GPU suite with the crash tracer and the per-test library watch.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS="rpw16 rpw24 rpw32 rpw20 rpw32t" TAG=r04i bash tools/gpu_ab_small.sh > /dev/null || exit 1
cut -c1-100 gpurun_out/r04/ab_small_r04i.log
TAG=r04i bash tools/gpu_suite_only.sh
