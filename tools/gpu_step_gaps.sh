# Launch gaps of a single-frame step (tools/step_gaps.py) at C2 and C3 from rocprofv3 kernel traces,
# for the product library and the libraries named in LIBS (tools/experiments/lib/libarx_<tag>.so);
# summaries under gpurun_out/$RD/step_gaps_<workload>_<lib>.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
RD=${RD:-r05}
O=gpurun_out/$RD
mkdir -p $O
for lib in prod notiming ${LIBS:-}; do
  T=1
  if [ "$lib" = prod ]; then L=""; elif [ "$lib" = notiming ]; then L=""; T=0; else L=$GRAFT_REPO_ROOT/tools/experiments/lib/libarx_$lib.so; fi
  for w in c2 c3; do
    STEP_GAPS_TIMING=$T ARX_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/$O/gaps_$w" -o run -- python3 tools/step_gaps.py run $w 40 > $O/gaps_$w.log 2>&1 || { tail -20 $O/gaps_$w.log; exit 1; }
    csv=$(find "$O/gaps_$w" -name '*kernel_trace.csv' | head -n 1)
    python3 tools/step_gaps.py analyze "$csv" 40 > $O/step_gaps_${w}_$lib.json || exit 1
    rm -rf "$O/gaps_$w"
    python3 -c "import json,sys; d=json.load(open('$O/step_gaps_${w}_$lib.json')); print('$w $lib span', d['span_us_median'], 'kernels', d['kernels_us_median'], 'between', d['between_kernels_us_median'], d['gap_before_us_median'])"
  done
done
