# GPU box: smoke, the whole -m gpu suite, the default bench, the layer-tail microbench.
# Usage: bash scripts/gpu_validate.sh TAG
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-val}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/pytest_gpu_$TAG.log 2>&1 && \
timeout -k 10 120 python scripts/sage_probe.py > gpurun_out/sage_$TAG.json 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?
echo "exit $rc"
[ $rc -eq 0 ] || exit $rc
# kernel stats of the same build (second pass; the bench above already exited 0)
mkdir -p /tmp/gnnprof && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gnnprof/prof -o run -- \
    python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-traffic > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
echo "prof exit $?"
find /tmp/gnnprof/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$TAG.csv \;
