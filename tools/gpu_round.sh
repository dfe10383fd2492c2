# smoke(), the default bench line and the GPU test suite (one process); logs under gpurun_out/$RD/.
# K= restricts pytest (-k expression); NOTEST=1 skips the suite.  The suite runs with pytest.s faulthandler
# and a native crash tracer (tools/run_gpu_suite.py), so a crash at any point (teardown included)
# leaves a trace.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r04}
O=gpurun_out/$RD
TAG=${TAG:-x}
mkdir -p $O
timeout -k 10 300 python -X faulthandler -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 || { echo "smoke failed"; tail -n 30 $O/smoke_$TAG.log; exit 1; }
tail -n 1 $O/smoke_$TAG.log
timeout -k 10 400 python3 bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err || { echo "bench failed"; tail -n 20 $O/bench_$TAG.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$TAG.json'));print(d['value'], d['ms_per_step'], d['phases_ms_rank0'], d['roofline']['frac'], d.get('moving_listener',{}).get('p50_ms'), d.get('moving_listener',{}).get('max_ms'))"
if [ -z "$NOTEST" ]; then
  timeout -k 10 900 python -u tools/run_gpu_suite.py tests -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"} > $O/pytest_gpu_$TAG.log 2>&1 || { echo "pytest failed"; tail -n 60 $O/pytest_gpu_$TAG.log; exit 1; }
  tail -n 3 $O/pytest_gpu_$TAG.log
fi
