# Per-kernel HBM traffic of the training step: two rocprofv3 counter passes (FETCH_SIZE, then
# WRITE_SIZE: they do not fit one pass) and one kernel-statistics pass over the same short bench,
# each in its own run and under its own time limit; scripts/pmc_table.py joins them.
#   bash scripts/pmc_kernels.sh TAG
set -o pipefail
TAG=$1
REPO=$(pwd)
mkdir -p gpurun_out
export TMPDIR=/tmp
export GNN_BENCH_GEMM_AB=0
ARGS="--steps 40 --warmup 5 --no-cpu-baseline --no-traffic --no-gpu-step --no-site-trace --no-roofline"
for C in FETCH_SIZE WRITE_SIZE; do
  echo "[pmc_kernels] $C ($(date +%T))"
  ( cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d /tmp/pmc_${TAG}_$C -o run -- \
      python -u $REPO/bench.py $ARGS > $REPO/gpurun_out/pmc_${TAG}_$C.json 2> $REPO/gpurun_out/pmc_${TAG}_$C.err ) || exit $?
  f=$(find /tmp/pmc_${TAG}_$C -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] || { echo "no counter CSV for $C"; exit 3; }
  python3 $REPO/scripts/pmc_table.py reduce "$f" $REPO/gpurun_out/pmc_${TAG}_$C.csv || exit $?
done
echo "[pmc_kernels] kernel stats ($(date +%T))"
( cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pmc_${TAG}_ks -o run -- \
    python -u $REPO/bench.py $ARGS > $REPO/gpurun_out/pmc_${TAG}_ks.json 2> $REPO/gpurun_out/pmc_${TAG}_ks.err ) || exit $?
find /tmp/pmc_${TAG}_ks -name "*kernel_stats.csv" -exec cp {} $REPO/gpurun_out/pmc_${TAG}_kstats.csv \;
python3 $REPO/scripts/pmc_table.py table $REPO/gpurun_out/pmc_${TAG}_FETCH_SIZE.csv $REPO/gpurun_out/pmc_${TAG}_WRITE_SIZE.csv \
    $REPO/gpurun_out/pmc_${TAG}_kstats.csv > $REPO/gpurun_out/pmc_${TAG}_table.md
cat $REPO/gpurun_out/pmc_${TAG}_table.md
