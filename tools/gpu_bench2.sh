set -o pipefail
cd "$GRAFT_REPO_ROOT"
TAG=ct K="convolution or bench or app" bash tools/gpu_tests.sh > gpurun_out/t_ct.txt; rc=$?; tail -3 gpurun_out/t_ct.txt; [ $rc = 0 ] || exit 1
for i in 1 2; do timeout -k 10 300 python bench.py --no-cpu-baseline --c5-frames 0 --steps 20 >> gpurun_out/b_ct.json 2>>gpurun_out/b_ct.err || exit 1; done
python -c "
import json
for l in open('gpurun_out/b_ct.json'):
    d=json.loads(l); print(d['ms_per_step'], d['phases_ms_rank0'], d['roofline_convolution']['frac'])"
