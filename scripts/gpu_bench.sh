# GPU box: bench (tiny sanity, then Reddit config 2), kernel microbench, rocprofv3 stats.
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --graph tiny --steps 5 --warmup 2 --no-cpu-baseline --batch-size 64 --samp-num 256 \
    > gpurun_out/bench_tiny.json 2> gpurun_out/bench_tiny.err && \
timeout -k 10 600 python bench.py --dump-batch /tmp/gnnprof/batch0.npz > gpurun_out/bench.json 2> gpurun_out/bench.err && \
timeout -k 10 300 python scripts/spmm_microbench.py /tmp/gnnprof/batch0.npz --out gpurun_out/micro.json \
    > gpurun_out/micro.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/gnnprof/prof -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err
rc=$?
find /tmp/gnnprof/prof -name "*stats*" -exec cp {} gpurun_out/ \; 2>/dev/null
ls -laR /tmp/gnnprof/prof > gpurun_out/prof_ls.txt 2>&1
echo "exit $rc"
