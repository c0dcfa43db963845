# N=2 rehearsal of the bench's multi-rank path with all ranks on the one GPU (gloo backend:
# RCCL refuses two ranks on one GPU): placement over 2 ranks, peer rows (both forms), the
# gradient exchange (both forms), max-over-ranks timing.
set -o pipefail
TAG=${1:-d2}
mkdir -p gpurun_out
export TMPDIR=/tmp
GNN_DIST_BACKEND=gloo timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 30 --warmup 5 --gpu-step-batches 15 \
    > gpurun_out/bench_dist2g_$TAG.json 2> gpurun_out/bench_dist2g_$TAG.err
rc=$?
echo "exit $rc"
exit $rc
