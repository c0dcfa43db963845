# Round-4 GPU pass i: the layer-2 forward with 16 nonzeros in flight (unit kernel, small tiles):
# spmm tests, the layer-2 forward sweep under rocprofv3, a short bench pair (U16 on / off).
set -o pipefail
TAG=${1:-r4i}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_spmm_gpu.py tests/test_abi.py tests/test_executor_gpu.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sw_$TAG -o run -- \
    python -u $REPO/scripts/spmm_l2fwd_sweep.py --out $REPO/gpurun_out/l2fwd_sweep_$TAG.json \
    > $REPO/gpurun_out/l2fwd_sweep_$TAG.log 2>&1 || exit 1
find /tmp/prof_sw_$TAG -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/kstats_l2fwd_$TAG.csv \;
cd $REPO
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  GNN_SPMM_SMALL_U16=$v timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_u16${v}_${TAG}_$i.json 2>> gpurun_out/bench_u16_$TAG.err || exit 1
done
echo "exit 0"
