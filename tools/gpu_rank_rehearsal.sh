# The one-GPU-per-process (RCCL rank) bench path under torch.distributed.run at one rank
# (--process-group), as the driver's N > 1 runs take it.  Output under gpurun_out/r03/.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r03
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --process-group --steps 10 --warmup 2 > gpurun_out/r03/bench_rank_rehearsal.json 2> gpurun_out/r03/bench_rank_rehearsal.err || { echo "rank bench failed"; tail -n 30 gpurun_out/r03/bench_rank_rehearsal.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/r03/bench_rank_rehearsal.json'));print(d['value'], d['n_gpus'], d['config']['parallelism'], d['runtime'])"
