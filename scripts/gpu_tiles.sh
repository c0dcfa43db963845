# GPU box: column-tile sweep of the aggregation kernel (GNN_SPMM_G / GNN_SPMM_NJ / GNN_SPMM_VW
# overrides) on a dumped Reddit LADIES batch. Usage: gpu_tiles.sh TAG "G NJ VW UNITS" ...
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
TAG=${1:-r1}
shift
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --dump-batch /tmp/gnnprof/batch0.npz \
    > /dev/null 2> gpurun_out/tiles_bench_$TAG.err || exit 1
timeout -k 10 300 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz --units 0 --reps 10 \
    > gpurun_out/tiles_${TAG}_default.log 2>&1 || exit 1
for cfg in "$@"; do
  set -- $cfg
  GNN_SPMM_G=$1 GNN_SPMM_NJ=$2 GNN_SPMM_VW=$3 timeout -k 10 300 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz \
      --units $4 --reps 10 > gpurun_out/tiles_${TAG}_g$1_nj$2_vw$3.log 2>&1 || exit 1
done
echo "exit 0"
