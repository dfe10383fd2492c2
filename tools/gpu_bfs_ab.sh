set -o pipefail
mkdir -p gpurun_out
for K in 1023 0 255 4095 16383 65535 10000000 1023; do
  echo "K=$K"
  ARX_BFS_K=$K timeout -k 10 120 python -u tools/trace_variants.py 921,921 || exit 1
done
