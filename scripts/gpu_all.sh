# GPU box: parity tests, smoke, bench (Reddit config 2), kernel microbench, rocprofv3 stats.
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py --dump-batch /tmp/gnnprof/batch0.npz > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz --units ${UNITS:-0,4,8,16,64,256} \
    --out gpurun_out/micro_$TAG.json > gpurun_out/micro_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gnnprof/prof -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-traffic --no-e2e > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?
find /tmp/gnnprof/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$TAG.csv \;
echo "exit $rc"
