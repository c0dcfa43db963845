# Round-4 GPU record + A/B in one call (the pool is congested): the whole GPU suite, smoke, the
# pre-split GEMM probe, A/B of the small-operand U = 16 unit kernel and the top layer's small
# products on the aux stream, the default bench (PMC traffic + CPU baseline), config 1 on the CPU,
# the self-launched N = 2 / 4 rehearsals (gloo, ranks sharing the one GPU), rocprofv3 stats.
set -o pipefail
TAG=${1:-r4k}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 1
timeout -k 10 200 python -u scripts/gemm_p3_probe.py --out gpurun_out/gemm_p3_$TAG.json > gpurun_out/gemm_p3_$TAG.log 2>&1
i=0
for cfg in "1 1" "0 1" "1 0" "1 1"; do
  set -- $cfg
  i=$((i+1))
  GNN_SPMM_SMALL_U16=$1 GNN_STEP_SMALL_OVERLAP=$2 timeout -k 10 200 python -u bench.py --steps 300 \
      --no-cpu-baseline --no-traffic > gpurun_out/bench_u$1_o$2_${TAG}_$i.json 2>> gpurun_out/bench_ab_$TAG.err || exit 1
done
timeout -k 10 400 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 1
timeout -k 10 200 python -u bench.py --cpu --steps 30 --warmup 3 > gpurun_out/bench_cpu_cfg1_$TAG.json \
    2> gpurun_out/bench_cpu_cfg1_$TAG.err || exit 1
GNN_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 2 --steps 20 --warmup 3 \
    > gpurun_out/bench_selflaunch2_$TAG.json 2> gpurun_out/bench_selflaunch2_$TAG.err || exit 1
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 300 --no-cpu-baseline --no-traffic > $REPO/gpurun_out/bench_prof_$TAG.json \
    2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
cd $REPO
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_$TAG.csv \; 2>/dev/null
[ $rc -eq 0 ] && GNN_DIST_BACKEND=gloo timeout -k 10 300 python3 bench.py --gpus 4 --steps 20 --warmup 3 \
    > gpurun_out/bench_selflaunch4_$TAG.json 2> gpurun_out/bench_selflaunch4_$TAG.err
rc=$?
echo "exit $rc"
exit $rc
