# Round 3: the end-to-end delta of the f32-input MFMA GEMM vs split3 on the default bench (A/B/A on
# one box), recorded once. Usage: TAG
set -o pipefail
TAG=${1:-g}
mkdir -p gpurun_out
for V in split3 f32 split3b; do
  ALGO=split3; [ "$V" = f32 ] && ALGO=f32
  GNN_GEMM_ALGO=$ALGO timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_gemm_${V}_$TAG.json 2> gpurun_out/bench_gemm_${V}_$TAG.err || { echo "failed $V"; exit 1; }
done
echo "exit 0"
