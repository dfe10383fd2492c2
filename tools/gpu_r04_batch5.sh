# Round-4 batch 5: smoke, bench and the GPU suite of the current build, then the guarded profile
# pass (rocprof kernel stats of the bench command, PMC traffic / state, lane counts) and the
# convolution's per-pass traffic.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=r04j bash tools/gpu_round.sh || exit 1
TAG=r04j bash tools/gpu_profile.sh || exit 1
bash tools/gpu_conv_pmc.sh
