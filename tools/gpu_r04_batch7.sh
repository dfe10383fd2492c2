# Round-4 batch 7: smoke, the default bench line (driver's K/W) and the GPU suite, then the C2 and C4
# workload lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r04
TAG=r04l bash tools/gpu_round.sh || exit 1
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_r04l_driverkw.json 2> $O/bench_r04l_driverkw.err || { tail -5 $O/bench_r04l_driverkw.err; exit 1; }
timeout -k 10 300 python3 bench.py --workload c2 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_c2_r04l.json 2> $O/bench_c2_r04l.err || { tail -5 $O/bench_c2_r04l.err; exit 1; }
timeout -k 10 400 python3 bench.py --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --c5-frames 0 > $O/bench_c4_r04l.json 2> $O/bench_c4_r04l.err || { tail -5 $O/bench_c4_r04l.err; exit 1; }
for f in bench_r04l_driverkw bench_c2_r04l bench_c4_r04l; do python3 -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['value'], d['ms_per_step'], d['phases_ms_rank0'], d.get('pipelined',{}).get('value'), d['preroll']['steps'])"; done
