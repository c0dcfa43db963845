# Prefetching SpMM walk vs the plain one (variant library built with -DGNN_SPMM_NOPF, loaded
# through GNN_SPMM_LIBRARY): per-call timings + output checksums, A/B/A; then the SpMM tests.
set -o pipefail
TAG=${1:-pf}
mkdir -p gpurun_out
for V in pf nopf pf; do
  if [ $V = nopf ]; then export GNN_SPMM_LIBRARY=$(pwd)/gnn_amd/libgnn_spmm_nopf.so; else unset GNN_SPMM_LIBRARY; fi
  QUICK=1 timeout -k 10 300 python -u scripts/spmm_ceiling.py >> gpurun_out/spmm_pf_$TAG.json 2>> gpurun_out/spmm_pf_$TAG.err || exit 1
  echo "--- $V" >> gpurun_out/spmm_pf_$TAG.json
done
unset GNN_SPMM_LIBRARY
timeout -k 10 500 python -u -m pytest tests/test_spmm_gpu.py tests/test_executor_gpu.py -m gpu -x -q --timeout 200 \
    --timeout-method thread > gpurun_out/gputest_spmm_pf_$TAG.log 2>&1 || exit 1
echo "exit 0"
