# Round-6 GPU batch: FIRST= test files run first (fail fast), then the rest of the GPU suite, in one
# process each (full-launch parity records into gpurun_out/$RD/full_launch_parity), then one default
# bench line.  TAG names the logs; K= restricts pytest (-k expression); NOBENCH=1 skips the bench,
# NOSUITE=1 the rest of the suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r06}
O=gpurun_out/$RD
TAG=${TAG:-x}
mkdir -p $O
export ARX_PARITY_RECORD=$O/full_launch_parity
suite() {  # $1 = log name, rest = pytest selection
    local log=$1; shift
    timeout -k 10 1000 python -u tools/run_gpu_suite.py "$@" -m gpu -x -v --timeout 300 --timeout-method thread \
        ${K:+-k "$K"} > $O/$log.log 2>&1
    local rc=$?
    tail -n 25 $O/$log.log
    return $rc
}
if [ -n "${FIRST:-}" ]; then
    suite pytest_gpu_${TAG}_first $FIRST || exit $?
fi
if [ -z "${NOSUITE:-}" ]; then
    ign=""
    for f in ${FIRST:-}; do ign="$ign --ignore=$f"; done
    suite pytest_gpu_$TAG tests $ign || exit $?
fi
[ -n "${NOBENCH:-}" ] && exit 0
timeout -k 10 300 python -u bench.py > $O/bench_$TAG.json 2> $O/bench_$TAG.err
rc=$?
tail -c 3000 $O/bench_$TAG.json
exit $rc
