# Pipeline / wave-state / memory counters of the trace kernel, one rocprofv3 --pmc pass per group
# (no trace domains), for each configuration in $CONFIGS: "prod" = the product libarx.so, "old" =
# tools/experiments/old (an older tree's package), anything else = tools/experiments/lib/libarx_<tag>.so.
# Output under gpurun_out/pmcs/v<tag>_<first counter>/; summarise with tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${CONFIGS:-prod}; do
  unset ARX_LIB ARX_PKG_ROOT
  if [ "$v" = old ]; then export ARX_PKG_ROOT=$R/tools/experiments/old
  elif [ "$v" != prod ]; then export ARX_LIB=$R/tools/experiments/lib/libarx_$v.so; fi
  for grp in ${GROUPS_OVERRIDE:-"GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
             "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
             "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
             "TA_TA_BUSY_sum TD_TD_BUSY_sum" \
             "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
             "TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum" \
             "TCC_HIT_sum TCC_MISS_sum"}; do
    tag=v${v}_$(echo $grp | cut -d' ' -f1)
    ARX_GUARD_OUT=$R/gpurun_out/pmcs/guard_$v.json timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmcs/$tag -o p -- python3 $R/tools/trace_once.py 2 > gpurun_out/pmcs/$tag.log 2>&1
    rc=$?
    echo "$tag rc=$rc" >> gpurun_out/pmcs/status.txt
    if [ $rc -ne 0 ]; then echo "pmc $tag failed rc=$rc"; tail -5 gpurun_out/pmcs/$tag.log; exit 1; fi
  done
done
python3 tools/pmc_summary.py gpurun_out/pmcs
