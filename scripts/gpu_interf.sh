# Interference of the staging stream with the step: gpu_step with the GPU extraction (default)
# vs the host extraction (no lx_* kernels beside the step; the CSR pieces travel in the blob).
set -o pipefail
TAG=${1:-if}
mkdir -p gpurun_out
i=0
for ARGS in "" "--host-extract" "" "--host-extract"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --steps 200 --no-cpu-baseline --no-traffic $ARGS \
      > gpurun_out/interf_${TAG}_$i.json 2> gpurun_out/interf_${TAG}_$i.err || exit 1
done
echo "exit 0"
