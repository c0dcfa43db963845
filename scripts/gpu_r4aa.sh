# Round-4 GPU pass aa: one row per combine workgroup for the 512-row layer-2 forward — SpMM tests,
# two benches, the per-dispatch trace.
set -o pipefail
TAG=${1:-r4aa}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py tests/test_executor_gpu.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
bash scripts/gpu_trace.sh $TAG
