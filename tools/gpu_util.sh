set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
timeout -k 10 300 python tools/trace_util.py > gpurun_out/util.log 2>&1 || { echo "util failed"; tail -20 gpurun_out/util.log; exit 1; }
cat gpurun_out/util.log
R=$GRAFT_REPO_ROOT
for v in 0 320; do
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" "TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TA_DATA_STALLED_BY_TC_CYCLES TA_TOTAL_WAVEFRONTS" "TD_TD_BUSY TD_TC_STALL TD_LOAD_WAVEFRONT TCP_PENDING_STALL_CYCLES" "TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum"; do
  tag=v${v}_$(echo $grp | cut -d' ' -f1)
  ARX_TRACE_KERNEL=$v timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc2/$tag -o p -- python3 $R/tools/trace_once.py 2 > gpurun_out/pmc2/$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc" >> gpurun_out/pmc2/status.txt
  if [ $rc -ne 0 ]; then echo "pmc $tag failed rc=$rc"; tail -5 gpurun_out/pmc2/$tag.log; exit 1; fi
done
done
echo pmc-done
