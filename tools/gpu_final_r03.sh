# Round-3 closing pass: the measurement pass (tools/gpu_profile_r03.sh), the A/B of the two
# round-3 trace changes against libraries built without them (tools/experiments/lib:
# nopool = -D ARX_TRACE_DYN_SHARE=0, nosign = -D ARX_TRACE_SIGNSEL=0), and the per-wave profile
# of C3 and C2 (libarx_prof).  Outputs under gpurun_out/r03/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03
TAG=${TAG:-r03e}
mkdir -p $O
TAG=$TAG bash tools/gpu_profile_r03.sh > $O/profile_pass_$TAG.log 2>&1 || { tail -20 $O/profile_pass_$TAG.log; exit 1; }
LIBS="prod nopool nosign" SHAPES="c3 c2" bash tools/gpu_ab_libs.sh > $O/ab_pool_signsel_$TAG.txt 2>&1 || { tail -20 $O/ab_pool_signsel_$TAG.txt; exit 1; }
for w in c3 c2; do
  ARX_LIB=tools/experiments/lib/libarx_prof.so timeout -k 10 120 python3 tools/trace_profile.py $w $O/trace_profile_$w.json > /dev/null || exit 1
done
cat $O/ab_pool_signsel_$TAG.txt
tail -3 $O/profile_pass_$TAG.log
