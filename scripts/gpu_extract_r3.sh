# Round 3: the one-pass LADIES extraction on the GPU box — parity tests, standalone probe, default
# bench (no PMC / CPU legs) and a rocprofv3 kernel-stats pass over a shorter bench.
# Usage: bash scripts/gpu_extract_r3.sh TAG
set -o pipefail
TAG=${1:-r3x}
mkdir -p gpurun_out
export TMPDIR=/tmp
REPO=$(pwd)
timeout -k 10 400 python -u -m pytest tests/test_extract.py tests/test_extract_full_gpu.py tests/test_native_loader.py \
    tests/test_executor_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/gputest_extract_$TAG.log 2>&1 && \
timeout -k 10 300 python -u scripts/extract_probe.py > gpurun_out/extract_probe_$TAG.json 2> gpurun_out/extract_probe_$TAG.err && \
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-traffic > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
    python -u $REPO/bench.py --steps 200 --no-cpu-baseline --no-traffic --no-gpu-step \
    > $REPO/gpurun_out/bench_prof_$TAG.json 2> $REPO/gpurun_out/bench_prof_$TAG.err
rc=$?
cd $REPO
find /tmp/prof_$TAG -name "*kernel_stats.csv" -exec cp {} gpurun_out/kstats_$TAG.csv \; 2>/dev/null
echo "exit $rc"
exit $rc
