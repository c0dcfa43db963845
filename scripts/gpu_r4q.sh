# Round-4 GPU pass q: the layer tails' dropout mask hashed per row (bit-identical) and one backward fork
# for the head + top-layer weight gradients, the split-row tail backward loading one row ahead: the fused /
# executor / model tests, two benches, the per-dispatch trace.
set -o pipefail
TAG=${1:-r4q}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_fused_gpu.py tests/test_executor_gpu.py tests/test_configs_gpu.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
bash scripts/gpu_trace.sh $TAG
