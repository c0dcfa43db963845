# Round-3 GPU box run: new parity tests first, then the whole GPU suite, smoke, default bench,
# and the config-1 CPU bench. Usage: bash scripts/gpu_r3.sh TAG [extra pytest -k expr]
set -o pipefail
TAG=${1:-r3}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err && \
timeout -k 10 300 python -u bench.py --cpu --steps 30 --warmup 3 > gpurun_out/bench_cpu_cfg1_$TAG.json \
    2> gpurun_out/bench_cpu_cfg1_$TAG.err
rc=$?
echo "exit $rc"
exit $rc
