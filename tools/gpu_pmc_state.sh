# Pipeline / wave-state counters of the trace kernel for the variants in $VARIANTS
# (default "0"), one rocprofv3 --pmc pass per group (no trace domains).  Output under
# gpurun_out/pmcs/<variant>_<first counter>/; summarise with tools/pmc_summary.py.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmcs
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in ${VARIANTS:-0}; do  # v: a tag (the library is ARX_LIB)
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM" \
           "SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_LDS" \
           "TA_TA_BUSY_sum TD_TD_BUSY_sum" \
           "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" \
           "TCC_HIT_sum TCC_MISS_sum"; do
  tag=v${v}_$(echo $grp | cut -d' ' -f1)
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmcs/$tag -o p -- python3 $R/tools/trace_once.py 1 > gpurun_out/pmcs/$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc" >> gpurun_out/pmcs/status.txt
  if [ $rc -ne 0 ]; then echo "pmc $tag failed rc=$rc"; tail -5 gpurun_out/pmcs/$tag.log; exit 1; fi
done
done
python3 tools/pmc_summary.py gpurun_out/pmcs
