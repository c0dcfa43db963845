# Round-4 GPU pass z: no stream wait on a staging event the host has already synchronized on —
# staging/extract tests, SKIP A/B/A/B under the bench (end to end and the driver's short form).
set -o pipefail
TAG=${1:-r4z}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_staging_gpu.py tests/test_extract.py tests/test_native_loader.py \
    tests/test_executor_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 \
    || { echo "tests failed"; exit 1; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  GNN_SKIP_SYNCED_WAIT=$v timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_skip${v}_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
  GNN_SKIP_SYNCED_WAIT=$v timeout -k 10 200 python3 bench.py --gpus 1 --steps 20 --warmup 5 \
      > gpurun_out/bench_s20_skip${v}_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
echo done
