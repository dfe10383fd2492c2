# Measurement pass on one MI355X: bench line, rocprofv3 kernel stats of the same command,
# PMC traffic (FETCH_SIZE / WRITE_SIZE, separate passes), pipeline state counters, the counting
# build's lane loads per query, and the guarded profile JSONs bench.py reads (tree hash + VGPRs).
# Outputs under gpurun_out/$RD/ (default r04).  TAG names the files.
# Build the counting library here first (it is not kept in the tree between rounds):
#   python -m audiorenderingv2_amd.build --exp count -D ARX_TRACE_COUNT=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=gpurun_out/${RD:-r04}
TAG=${TAG:-r04}
mkdir -p $O
timeout -k 10 400 python3 bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -20 $O/bench_$TAG.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_$TAG -o run -- python3 bench.py --frames-in-flight 1 --no-cpu-baseline --c5-frames 0 --no-streaming > $O/prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof_$TAG.log; exit 1; }
mkdir -p $O/pmc_traffic_$TAG
for grp in FETCH_SIZE WRITE_SIZE TCC_EA0_RDREQ_sum; do
  ARX_GUARD_OUT=$R/$O/guard_traffic.json timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/$O/pmc_traffic_$TAG/$grp -o p -- python3 tools/trace_once.py 2 > $O/pmc_traffic_$TAG/$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 $O/pmc_traffic_$TAG/$grp.log; exit 1; }
done
python3 tools/make_traffic.py $O/pmc_traffic_$TAG c3 $O/trace_traffic.json $O/guard_traffic.json || exit 1
rm -rf gpurun_out/pmcs
CONFIGS=prod bash tools/gpu_pmc_state.sh > $O/pmc_state_$TAG.txt 2>&1 || { echo "pmc state failed"; tail -20 $O/pmc_state_$TAG.txt; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcs $O/trace_td_c3.json gpurun_out/pmcs/guard_prod.json > /dev/null || exit 1
ARX_LIB=tools/experiments/lib/libarx_count.so timeout -k 10 120 python3 tools/trace_counts.py > $O/trace_counts_c3.json || exit 1
python3 tools/vmem_ceiling.py profiles/r02/td_microbench_sizes.txt $O/pmc_state_$TAG.txt $O/trace_counts_c3.json gpurun_out/pmcs/guard_prod.json > $O/trace_vmem_ceiling.json || exit 1
cat $O/trace_traffic.json $O/trace_td_c3.json $O/trace_counts_c3.json
python3 -c "import json;d=json.load(open('$O/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['frac'])"
