# Stream form of the aggregation (spmm_stream_kernel, GNN_SPMM_STREAM=1, U = GNN_SPMM_SU) vs the
# unit form: per-call timings on the real operands (scripts/spmm_ceiling.py, QUICK=1), A/B/A,
# then the SpMM GPU tests with the stream form forced on.
set -o pipefail
TAG=${1:-st}
mkdir -p gpurun_out
for V in "0 4" "1 4" "1 8" "0 4" "1 4"; do
  set -- $V
  GNN_SPMM_STREAM=$1 GNN_SPMM_SU=$2 QUICK=1 timeout -k 10 300 python -u scripts/spmm_ceiling.py \
      >> gpurun_out/spmm_stream_$TAG.json 2>> gpurun_out/spmm_stream_$TAG.err || exit 1
  echo "--- stream=$1 su=$2" >> gpurun_out/spmm_stream_$TAG.json
done
GNN_SPMM_STREAM=1 timeout -k 10 500 python -u -m pytest tests/test_spmm_gpu.py tests/test_torch_ext.py -m gpu -x -q \
    --timeout 200 --timeout-method thread > gpurun_out/gputest_spmm_stream_$TAG.log 2>&1 || exit 1
echo "exit 0"
