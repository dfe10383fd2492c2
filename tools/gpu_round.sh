# GPU test suite (one process), smoke() and the default bench line; logs under gpurun_out/$RD/.
# K= restricts pytest (-k expression); NOTEST=1 skips the suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r04}
O=gpurun_out/$RD
TAG=${TAG:-x}
mkdir -p $O
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -n 40 $O/pytest_gpu_$TAG.log; exit 1; }
  tail -n 2 $O/pytest_gpu_$TAG.log
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -n 20 $O/smoke_$TAG.log; exit 1; }
tail -n 1 $O/smoke_$TAG.log
timeout -k 10 400 python3 bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -n 20 $O/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['frac'], d.get('moving_listener',{}).get('p50_ms'), d.get('moving_listener',{}).get('max_ms'))"
