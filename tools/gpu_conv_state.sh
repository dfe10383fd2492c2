# Instruction / wait-state counters per convolution pass (C3 file convolution), one rocprofv3 --pmc pass.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/conv_state
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VMEM GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/conv_state/s -o p -- python3 $R/tools/conv_once.py 3 > gpurun_out/conv_state/s.log 2>&1 || { tail -5 gpurun_out/conv_state/s.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FP64 SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --output-format csv -d $R/gpurun_out/conv_state/t -o p -- python3 $R/tools/conv_once.py 3 > gpurun_out/conv_state/t.log 2>&1 || { tail -5 gpurun_out/conv_state/t.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
per = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/conv_state/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Kernel_Name"].replace("void ", "").replace("arx::(anonymous namespace)::", "").split("(")[0]
        if "pass" in n:
            per[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, d in sorted(per.items()):
    print(n, {k: round(sum(v) / len(v)) for k, v in sorted(d.items())})
PY
