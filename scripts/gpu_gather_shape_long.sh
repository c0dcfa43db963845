set -o pipefail
mkdir -p gpurun_out
for K in 4096 15740 22176; do for G in 8 16 32; do for U in 4 8; do
  PER_WAVE=1024 timeout -k 10 60 scripts/bin/gather_shape $K $G $U >> gpurun_out/gather_shape4.json || exit 1
done; done; done
echo "exit 0"
