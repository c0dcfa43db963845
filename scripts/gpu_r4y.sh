# Round-4 GPU pass y: the clip factor computed inside the Adam launch (gnn_adam_clip_f32) — optimizer,
# executor and distributed tests, two benches, the per-dispatch trace.
set -o pipefail
TAG=${1:-r4y}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_optim_gpu.py tests/test_executor_gpu.py tests/test_dist_gpu.py \
    -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 \
    || { echo "tests failed"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
bash scripts/gpu_trace.sh $TAG
