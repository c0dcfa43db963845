# Round-4 GPU pass t (u: rem <= 32, 4 pieces): split3 tail tiles (k pieces for the last partial round) — GEMM + executor +
# fused tests, the tile probe with the tail on, TAIL A/B/A/B under the bench, the trace.
set -o pipefail
TAG=${1:-r4t}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_executor_gpu.py tests/test_fused_gpu.py \
    tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 \
    || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -u scripts/gemm_tiles_probe.py --out gpurun_out/gemm_tiles_$TAG.json > gpurun_out/gemm_tiles_$TAG.log 2>&1 || exit 1
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  GNN_GEMM_TAIL=$v timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_tail${v}_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
bash scripts/gpu_trace.sh $TAG
