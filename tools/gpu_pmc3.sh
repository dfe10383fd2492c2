set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 320; do
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD" "SQ_INST_LEVEL_VMEM SQ_ACCUM_PREV_HIRES" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum" "TA_DATA_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum" "TCC_HIT_sum TCC_MISS_sum TCC_BUSY_sum"; do
  tag=v${v}_$(echo $grp | cut -d' ' -f1)
  ARX_TRACE_KERNEL=$v timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc3/$tag -o p -- python3 $R/tools/trace_once.py 1 > gpurun_out/pmc3/$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc" >> gpurun_out/pmc3/status.txt
  if [ $rc -ne 0 ]; then echo "pmc $tag failed rc=$rc"; tail -5 gpurun_out/pmc3/$tag.log; exit 1; fi
done
done
echo pmc-done
