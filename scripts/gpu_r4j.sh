# Round-4 GPU pass j: spmm / executor tests; the pre-split (p3) GEMM probe; the layer-2 forward sweep under rocprofv3; bench A/B of
# the small-operand U = 16 unit kernel (GNN_SPMM_SMALL_U16) and the top layer's small products on
# the aux stream (GNN_STEP_SMALL_OVERLAP), interleaved; rocprofv3 stats of the default bench.
set -o pipefail
TAG=${1:-r4j}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_spmm_gpu.py tests/test_abi.py tests/test_executor_gpu.py \
    tests/test_fused_gpu.py tests/test_configs_gpu.py tests/test_dist_gpu.py -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -u scripts/gemm_p3_probe.py --out gpurun_out/gemm_p3_$TAG.json > gpurun_out/gemm_p3_$TAG.log 2>&1 \
    || { echo "p3 probe failed"; exit 1; }
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_sw_$TAG -o run -- \
    python -u $REPO/scripts/spmm_l2fwd_sweep.py --out $REPO/gpurun_out/l2fwd_sweep_$TAG.json \
    > $REPO/gpurun_out/l2fwd_sweep_$TAG.log 2>&1 || exit 1
find /tmp/prof_sw_$TAG -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/kstats_l2fwd_$TAG.csv \;
cd $REPO
i=0
for rep in 1 2; do
  for cfg in "1 1" "0 1" "1 0"; do
    set -- $cfg
    i=$((i+1))
    GNN_SPMM_SMALL_U16=$1 GNN_STEP_SMALL_OVERLAP=$2 timeout -k 10 300 python -u bench.py --steps 300 \
        --no-cpu-baseline --no-traffic > gpurun_out/bench_u$1_o$2_${TAG}_$i.json 2>> gpurun_out/bench_ab_$TAG.err || exit 1
  done
done
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 200 --no-cpu-baseline --no-traffic > $REPO/gpurun_out/bench_prof_$TAG.json \
    2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/kstats_$TAG.csv \;
echo "exit $rc"
exit $rc
