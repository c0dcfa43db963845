# GPU box: bench with hipBLASLt (default) vs rocBLAS for the dense fp32 GEMMs.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r1}
timeout -k 10 600 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/blas_lt_$TAG.json 2> gpurun_out/blas_lt_$TAG.err && \
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 600 python bench.py --no-cpu-baseline --no-traffic > gpurun_out/blas_roc_$TAG.json 2> gpurun_out/blas_roc_$TAG.err
echo "exit $?"
