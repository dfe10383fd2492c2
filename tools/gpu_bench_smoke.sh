# smoke() and the default bench line (guarded profile fields included when they match); TAG names the files.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
TAG=${TAG:-x}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -n 20 gpurun_out/r03/smoke_$TAG.log; exit 1; }
tail -n 1 gpurun_out/r03/smoke_$TAG.log
timeout -k 10 400 python3 bench.py > gpurun_out/r03/bench_$TAG.json 2> gpurun_out/r03/bench_$TAG.err || { echo "bench failed"; tail -n 20 gpurun_out/r03/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], (d.get('roofline_valu') or {}).get('frac'), (d.get('roofline_td') or {}).get('frac'))"
