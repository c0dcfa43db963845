# Wide-row tile rule (F >= 1024: 128-float tiles as 16-lane groups x 2 chunks) vs the round-3 choice
# (GNN_SPMM_TILES=0): SpMM GPU tests, then A/B/A/B default bench runs (500 steps) with per-call-site
# HIP-event timings.
set -o pipefail
TAG=${TAG:-ta}
mkdir -p gpurun_out/tiles_$TAG
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py tests/test_executor_gpu.py tests/test_fused_gpu.py -m gpu -x -q \
    --timeout 120 --timeout-method thread > gpurun_out/tiles_$TAG/tests.log 2>&1 || { echo "tests failed"; exit 1; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  GNN_SPMM_TILES=$v timeout -k 10 300 python -u bench.py --steps 500 --no-cpu-baseline --no-traffic \
      > gpurun_out/tiles_$TAG/bench_${i}_t$v.json 2> gpurun_out/tiles_$TAG/bench_${i}_t$v.err || exit 1
done
echo "exit 0"
