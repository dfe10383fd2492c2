# Round-5 bench lines on the final tree: the default bench (driver's K / W), its rocprofv3 kernel
# stats and the kernel-times leg's agreement (tools/trace_legs.py), C2 and C4 lines, smoke.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r05
TAG=${TAG:-r05j}
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { tail -5 $O/bench_$TAG.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof_$TAG" -o run -- python3 bench.py > $O/bench_${TAG}_under_rocprof.json 2> $O/prof_$TAG.log || { tail -20 $O/prof_$TAG.log; exit 1; }
stats=$(find $O/prof_$TAG -name '*kernel_stats.csv' | head -n 1)
trace=$(find $O/prof_$TAG -name '*kernel_trace.csv' | head -n 1)
cp "$stats" $O/bench_${TAG}_kernel_stats.csv
python3 tools/trace_legs.py "$trace" $O/bench_${TAG}_under_rocprof.json > $O/trace_legs_$TAG.json || exit 1
rm -rf $O/prof_$TAG
timeout -k 10 300 python bench.py --workload c2 > $O/bench_c2_$TAG.json 2> $O/bench_c2_$TAG.err || { tail -5 $O/bench_c2_$TAG.err; exit 1; }
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 > $O/bench_c4_$TAG.json 2> $O/bench_c4_$TAG.err || { tail -5 $O/bench_c4_$TAG.err; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke_$TAG.txt 2>&1 || { tail -20 $O/smoke_$TAG.txt; exit 1; }
python3 - <<PY
import json
for f in ("bench_$TAG", "bench_c2_$TAG", "bench_c4_$TAG"):
    d = json.loads([l for l in open(f"$O/{f}.json") if l.startswith("{")][-1])
    sf = d.get("single_frame") or {}
    print(f, d["value"], d["ms_per_step"], sf.get("value"), d["kernel_times_leg"]["ms_per_step"], d["phases_ms_rank0"])
print(json.load(open("$O/trace_legs_$TAG.json")))
PY
tail -1 $O/smoke_$TAG.txt
