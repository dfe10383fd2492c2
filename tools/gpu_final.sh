# Round-end GPU evidence: the full round (tests, bench, rocprof, PMC) + smoke + the C2 / C4 bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=${TAG:-final}
bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py --workload c2 > gpurun_out/bench_c2_$TAG.json 2> gpurun_out/bench_c2_$TAG.err || { tail -5 gpurun_out/bench_c2_$TAG.err; exit 1; }
timeout -k 10 400 python bench.py --workload c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_$TAG.json 2> gpurun_out/bench_c4_$TAG.err || { tail -5 gpurun_out/bench_c4_$TAG.err; exit 1; }
python - <<PY
import json
for w in ("c2", "c4"):
    d = json.load(open(f"gpurun_out/bench_{w}_$TAG.json"))
    print(w, d["value"], d["ms_per_step"], d["phases_ms_rank0"], d["roofline"]["frac"])
PY
