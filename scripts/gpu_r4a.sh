# Round-4 first GPU pass: the GPU suite, smoke, the self-launched N = 2 rehearsal (both ranks on
# the one GPU over gloo, no torchrun on the command line), the extraction-check A/B, and the
# papers-shaped run with --locality-sampling.
# Usage: bash scripts/gpu_r4a.sh TAG
set -o pipefail
TAG=${1:-r4a}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_$TAG.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 && \
GNN_DIST_BACKEND=gloo timeout -k 10 400 python3 bench.py --gpus 2 --steps 10 --warmup 3 \
    > gpurun_out/bench_selflaunch2_$TAG.json 2> gpurun_out/bench_selflaunch2_$TAG.err && \
GNN_EXTRACT_CHECK=step timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
    > gpurun_out/bench_xcheck_step_$TAG.json 2> gpurun_out/bench_xcheck_step_$TAG.err && \
GNN_EXTRACT_CHECK=end timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
    > gpurun_out/bench_xcheck_end_$TAG.json 2> gpurun_out/bench_xcheck_end_$TAG.err && \
GNN_EXTRACT_CHECK=step timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
    > gpurun_out/bench_xcheck_step2_$TAG.json 2> gpurun_out/bench_xcheck_step2_$TAG.err && \
timeout -k 10 400 python -u bench.py --graph papers --locality-sampling --steps 100 --no-cpu-baseline --no-traffic \
    > gpurun_out/bench_papers_locality_$TAG.json 2> gpurun_out/bench_papers_locality_$TAG.err
rc=$?
echo "exit $rc"
exit $rc
