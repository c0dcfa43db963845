# Round-4 GPU pass r: non-temporal X0 staging gathers — staging tests, NT A/B/A/B under the bench,
# the per-dispatch trace with NT on.
set -o pipefail
TAG=${1:-r4r}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_staging_gpu.py tests/test_spmm_gpu.py -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/gputest_$TAG.log 2>&1 || { echo "tests failed"; exit 1; }
i=0
for v in 1 0 1 0; do
  i=$((i+1))
  GNN_GATHER_NT=$v timeout -k 10 300 python -u bench.py --steps 300 --no-cpu-baseline --no-traffic \
      > gpurun_out/bench_nt${v}_${TAG}_$i.json 2>> gpurun_out/bench_$TAG.err || exit 1
done
bash scripts/gpu_trace.sh $TAG
