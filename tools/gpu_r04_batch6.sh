# Round-4 batch 6: cache-policy bits of the trace kernel's loads (triangles nt / sc0 / sc1, nodes nt)
# against the product, on C2, one 8-GPU rank's C5 shard and C3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
LIBS="trint trisc0 trisc1 nodent" TAG=r04k bash tools/gpu_ab_small.sh > /dev/null || exit 1
cut -c1-150 gpurun_out/r04/ab_small_r04k.log
