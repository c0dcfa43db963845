# GPU box: dump one batch via a short bench run, then the per-call-site SpMM sweep.
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
TAG=${1:-r1}
timeout -k 10 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --dump-batch /tmp/gnnprof/batch0.npz \
    > /dev/null 2> gpurun_out/micro_bench_$TAG.err && \
timeout -k 10 300 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz --units ${UNITS:-0,64,128,256,512,1024} \
    --out gpurun_out/micro_$TAG.json > gpurun_out/micro_$TAG.log 2>&1
echo "exit $?"
