# Per-workgroup phases of the C3 convolution (tools/conv_phases.py, measurement build libarx_cprof.so)
# and the standalone per-pass kernel times (rocprofv3) of the product library; outputs under
# gpurun_out/$RD/.
# Build it here first: python -m audiorenderingv2_amd.build --exp cprof -D ARX_CONV_PROF=1
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
RD=${RD:-r04}
O=gpurun_out/$RD
TAG=${TAG:-x}
mkdir -p $O
ARX_LIB=${ARX_LIB:-tools/experiments/lib/libarx_cprof.so} timeout -k 10 240 python3 tools/conv_phases.py 6 $O/conv_phases_$TAG.json > $O/conv_phases_$TAG.log 2>&1 || { echo "conv_phases failed"; tail -n 20 $O/conv_phases_$TAG.log; exit 1; }
python3 -c "
import json; d=json.load(open('$O/conv_phases_$TAG.json')); print('window', round(d['conv_window_us'],1))
for k,p in d['passes'].items(): print(k, {q: (round(v,2) if isinstance(v,float) else [round(x,2) for x in v] if isinstance(v,list) else v) for q,v in p.items()})"
