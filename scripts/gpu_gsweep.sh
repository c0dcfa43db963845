# Column-tile width sweep of the aggregation on the step's real call shapes (scripts/spmm_ceiling.py
# QUICK=1): the default choice vs forced lane groups G = 16 / 32 / 64 (64 / 128 / 256-float tiles).
set -o pipefail
TAG=${1:-gs}
mkdir -p gpurun_out/gsweep_$TAG
export TMPDIR=/tmp
QUICK=1 timeout -k 10 240 python3 -u scripts/spmm_ceiling.py > gpurun_out/gsweep_$TAG/default.jsonl 2> gpurun_out/gsweep_$TAG/default.err || exit 1
for G in 16 32 64; do
  GNN_SPMM_G=$G GNN_SPMM_NJ=1 QUICK=1 timeout -k 10 240 python3 -u scripts/spmm_ceiling.py \
      > gpurun_out/gsweep_$TAG/g$G.jsonl 2> gpurun_out/gsweep_$TAG/g$G.err || exit 1
done
QUICK=1 timeout -k 10 240 python3 -u scripts/spmm_ceiling.py > gpurun_out/gsweep_$TAG/default2.jsonl 2> gpurun_out/gsweep_$TAG/default2.err || exit 1
echo "exit 0"
