# Round-4 GPU pass w: the split3 split with packed subtractions (v_pk_add_f32, 144 vs 159 VALU per
# two k tiles) against the previous build (variants/libgnn_spmm_base.so via GNN_SPMM_LIBRARY):
# GEMM + executor tests, the layer GEMM microbench for both, bench A/B/A/B.
set -o pipefail
TAG=${1:-r4w}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_executor_gpu.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -u scripts/gemm_bench.py > gpurun_out/gemm_bench_new_$TAG.log 2>&1 || exit 1
GNN_SPMM_LIBRARY=$(pwd)/variants/libgnn_spmm_base.so timeout -k 10 200 python -u scripts/gemm_bench.py \
    > gpurun_out/gemm_bench_base_$TAG.log 2>&1 || exit 1
i=0
for v in new base new base; do
  i=$((i+1))
  if [ $v = base ]; then L=$(pwd)/variants/libgnn_spmm_base.so; else L=$(pwd)/gnn_amd/libgnn_spmm.so; fi
  GNN_SPMM_LIBRARY=$L timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_${v}_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
echo done
