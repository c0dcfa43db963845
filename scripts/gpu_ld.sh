# GPU box: layer-0 aggregation vs X0 row stride / column tile shape (microbench on a dumped batch).
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
export TMPDIR=/tmp
TAG=${1:-ld}
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-e2e \
    --dump-batch /tmp/gnnprof/batch0.npz > gpurun_out/dump_$TAG.json 2> gpurun_out/dump_$TAG.err || exit 1
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz --units 256 --layers 0 \
      --f0 "602:604,602:608,602:640,640" --out gpurun_out/micro_${TAG}_$name.json > gpurun_out/micro_${TAG}_$name.log 2>&1
}
run default && run g16nj2 GNN_SPMM_G=16 GNN_SPMM_NJ=2 && run g32 GNN_SPMM_G=32 GNN_SPMM_NJ=1 && \
run g8 GNN_SPMM_G=8 GNN_SPMM_NJ=1
echo "exit $?"
