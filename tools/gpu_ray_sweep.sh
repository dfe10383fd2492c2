set -e
mkdir -p gpurun_out/r06
for R in 100,100,100 200,100,100 400,100,100 1000,100,100; do
  RAYS=$R timeout -k 10 120 python tools/trace_once.py 9 >> gpurun_out/r06/ray_sweep.txt
done
RAYS=100,100,100 BOUNCES=32 timeout -k 10 120 python tools/trace_once.py 9 >> gpurun_out/r06/ray_sweep.txt
RAYS=1000,100,100 BOUNCES=32 timeout -k 10 120 python tools/trace_once.py 5 >> gpurun_out/r06/ray_sweep.txt
cat gpurun_out/r06/ray_sweep.txt
