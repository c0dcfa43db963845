# A/B of a variant SpMM library (built with a -D switch into gnn_amd/libgnn_spmm_<name>.so,
# loaded through GNN_SPMM_LIBRARY) against the in-tree one: per-call timings and output
# checksums on the real operands (scripts/spmm_ceiling.py, QUICK=1), A/B/A/B. Usage: TAG NAME
set -o pipefail
TAG=${1:-v}
NAME=${2:-variant}
mkdir -p gpurun_out
for V in main alt main alt; do
  if [ $V = alt ]; then export GNN_SPMM_LIBRARY=$(pwd)/gnn_amd/libgnn_spmm_$NAME.so; else unset GNN_SPMM_LIBRARY; fi
  QUICK=1 timeout -k 10 300 python -u scripts/spmm_ceiling.py >> gpurun_out/spmm_ab_$TAG.json 2>> gpurun_out/spmm_ab_$TAG.err || exit 1
  echo "--- $V" >> gpurun_out/spmm_ab_$TAG.json
done
echo "exit 0"
