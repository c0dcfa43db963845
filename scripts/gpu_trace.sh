# rocprofv3 kernel trace of a short default bench (no PMC): the per-kernel start/end on each
# queue, copied (gzip) into gpurun_out/ for the compute-stream gap analysis (scripts/trace_gaps.py).
set -o pipefail
TAG=${1:-tr}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/trace_$TAG -o run -- \
    python -u $REPO/bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-traffic --no-roofline --no-gpu-step \
    > $REPO/gpurun_out/bench_trace_$TAG.json 2> $REPO/gpurun_out/bench_trace_$TAG.err
rc=$?
cd $REPO
f=$(find /tmp/trace_$TAG -name "*kernel_trace.csv" | head -1)
[ -n "$f" ] && gzip -c "$f" > gpurun_out/kernel_trace_$TAG.csv.gz
echo "exit $rc"
exit $rc
