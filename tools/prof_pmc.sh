set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCC_EA0_RDREQ_sum"; do
  tag=$(echo $grp | cut -d' ' -f1)
  timeout -k 10 180 rocprofv3 --pmc $grp --output-format csv -d $R/gpurun_out/pmc/$tag -o p -- python3 $R/tools/trace_once.py 2 > gpurun_out/pmc/$tag.log 2>&1
  echo "$tag rc=$?" >> gpurun_out/pmc/status.txt
done
