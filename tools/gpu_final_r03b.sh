# Round-3 closing measurement pass of the final trace kernel: bench line + rocprofv3 kernel stats +
# PMC traffic / pipeline state / lane-load counts / vector-memory mix (tools/gpu_profile_r03.sh, the
# guarded profile JSONs bench.py reads), C2 and C4 bench lines, and the per-wave profile of C3.
# Outputs under gpurun_out/r03/; TAG names the files.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r03
TAG=${TAG:-r03m}
mkdir -p $O
TAG=$TAG bash tools/gpu_profile_r03.sh > $O/profile_pass_$TAG.log 2>&1 || { tail -n 20 $O/profile_pass_$TAG.log; exit 1; }
tail -n 3 $O/profile_pass_$TAG.log
for w in c2 c4; do
  timeout -k 10 400 python3 bench.py --workload $w --c5-frames 0 > $O/bench_${w}_$TAG.json 2> $O/bench_${w}_$TAG.err || { echo "bench $w failed"; tail -n 20 $O/bench_${w}_$TAG.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_${w}_$TAG.json'));print('$w', d['value'], d['ms_per_step'], d['phases_ms_rank0'])"
done
ARX_LIB=tools/experiments/lib/libarx_prof.so timeout -k 10 120 python3 tools/trace_profile.py c3 $O/trace_profile_c3.json > /dev/null || exit 1
