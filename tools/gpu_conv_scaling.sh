# File-convolution time against the number of block pairs (C3 plan, 48 kHz, n = 96 000): the
# event-window time of tools/conv_once.py for 1, 2, 4 and 8.4 pairs, and a rocprof kernel-stats
# summary per size.  Output under gpurun_out/r03/conv_scaling/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r03/conv_scaling
mkdir -p $O
for f in 96000 192000 384000 807498; do
  CONV_FRAMES=$f timeout -k 10 120 python3 tools/conv_once.py 8 || exit 1
  CONV_FRAMES=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/f$f -o run -- python3 tools/conv_once.py 8 > $O/f$f.log 2>&1 || exit 1
done
for f in 96000 192000 384000 807498; do
  echo "== $f"; python3 -c "
import csv,glob
for r in csv.DictReader(open(glob.glob('$O/f$f/**/run_kernel_stats.csv', recursive=True)[0])):
    if 'pass_' in r['Name']: print(r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs'])/1e3,2))
"
done
