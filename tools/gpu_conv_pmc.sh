# FETCH_SIZE / WRITE_SIZE per convolution pass (C3 file convolution), one rocprofv3 --pmc pass each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/conv_pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/conv_pmc/stats -o p -- python3 $R/tools/conv_once.py 5 > gpurun_out/conv_pmc/stats.log 2>&1 || { tail -5 gpurun_out/conv_pmc/stats.log; exit 1; }
for grp in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/conv_pmc/$grp -o p -- python3 $R/tools/conv_once.py 3 > gpurun_out/conv_pmc/$grp.log 2>&1 || { echo "pmc $grp failed"; tail -5 gpurun_out/conv_pmc/$grp.log; exit 1; }
done
python3 tools/conv_pmc_summary.py gpurun_out/conv_pmc
