set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-traffic --no-e2e --dump-batch /tmp/gnnprof/batch0.npz > /dev/null 2>&1 || exit 1
for g in 0 16 32; do
  if [ $g = 0 ]; then E=""; else E="GNN_SPMM_G=$g GNN_SPMM_NJ=1"; fi
  env $E timeout -k 10 120 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz --units 128,256 --layers 1,2 > gpurun_out/l1bwd_g$g.log 2>&1 || exit 1
done
