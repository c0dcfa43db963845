# GPU box: rocprofv3 kernel-trace summary of the benchmark (csv), copied into gpurun_out/.
set -o pipefail
mkdir -p gpurun_out /tmp/gnnprof
export TMPDIR=/tmp
TAG=${1:-r1}
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/gnnprof/prof -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_prof_$TAG.json 2> gpurun_out/bench_prof_$TAG.err
rc=$?
find /tmp/gnnprof/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats_$TAG.csv \;
ls -laR /tmp/gnnprof/prof > gpurun_out/prof_ls.txt 2>&1
echo "exit $rc"
